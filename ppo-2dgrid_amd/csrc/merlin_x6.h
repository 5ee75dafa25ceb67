// merlin_x6.h -- the exact three-plane bf16 form of fp32 values used by fc1's matrix-core GEMMs
// (merlin_gemm.hip): x = x0 + x1 + x2 with x0 = bf16(x), x1 = bf16(x - x0), x2 = bf16(x - x0 - x1)
// (round to nearest; every subtraction is exact in fp32 and each plane takes the next 8 of the 24
// significand bits, so the planes add back to x exactly for every finite |x| >= 2^-110, where the
// third plane is still a normal number; below that bits under 2^-126 absolute may be lost).
//
// Layout of a row-major fp32 matrix X[R][C] (C % 8 == 0) in planes: bf16 [R][C/8][3][8] -- per
// group of 8 consecutive values three 16-B chunks, planes 0, 1, 2.  Flat float4 number q4 of X is
// half q4 & 1 of group q4 >> 1.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace merlin {

__device__ __forceinline__ uint32_t x6_pack2(float a, float b) {
    const __bf16 ha = (__bf16)a, hb = (__bf16)b;
    return (uint32_t)__builtin_bit_cast(uint16_t, ha) | ((uint32_t)__builtin_bit_cast(uint16_t, hb) << 16);
}
__device__ __forceinline__ float x6_lo(uint32_t p) { return __uint_as_float(p << 16); }
__device__ __forceinline__ float x6_hi(uint32_t p) { return __uint_as_float(p & 0xffff0000u); }

// planes of 4 consecutive values: out[p] = plane p, value 0 in the low half of .x
__device__ __forceinline__ void x6_split4(const float4 v, uint2 out[3]) {
    uint32_t a = x6_pack2(v.x, v.y), b = x6_pack2(v.z, v.w);
    out[0] = make_uint2(a, b);
    float rx = v.x - x6_lo(a), ry = v.y - x6_hi(a), rz = v.z - x6_lo(b), rw = v.w - x6_hi(b);
    a = x6_pack2(rx, ry);
    b = x6_pack2(rz, rw);
    out[1] = make_uint2(a, b);
    rx -= x6_lo(a);
    ry -= x6_hi(a);
    rz -= x6_lo(b);
    rw -= x6_hi(b);
    out[2] = make_uint2(x6_pack2(rx, ry), x6_pack2(rz, rw));
}

// store the planes of flat float4 number q4 (planes as uint2 units: 6 per group of 8 values)
__device__ __forceinline__ void x6_store4(uint2 *__restrict__ planes, int64_t q4, const float4 v) {
    uint2 p[3];
    x6_split4(v, p);
    uint2 *d = planes + (q4 >> 1) * 6 + (q4 & 1);
    d[0] = p[0];
    d[2] = p[1];
    d[4] = p[2];
}

}  // namespace merlin
