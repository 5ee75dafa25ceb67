"""CPU: every roofline of the bench line finds its HBM traffic in the committed PMC passes (bench.py pmc_traffic),
and only in passes at least as new as the newest kernel trace -- a stale alias or an outdated pass would silently
report another kernel's bytes (round-5 verdict)."""
import glob
import importlib.util
import json
import os

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def bench():
    spec = importlib.util.spec_from_file_location("bench_under_test", os.path.join(REPO, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def newest_tag():
    stats = sorted(glob.glob(os.path.join(REPO, "profiles", "*_kernel_stats.md")))
    return os.path.basename(stats[-1]).split("_")[0]


# the spans bench.py's loop times by default (merlin._native.KernelTimer) that carry a roofline with traffic
SPANS = ["gemm_fc1_fwd", "gemm_fc1_dgrad", "gemm_wgrad", "gemm_window_fwd", "k_seg_sum_R", "k_seg_sum_S",
         "k_seg_sum_dQ", "k_seg_sum_dT2", "k_head_bwd", "k_window_conv3", "k_heads_fwd", "gemm_rollout_fc1",
         "k_act_heads", "k_window_lut"]


@pytest.mark.parametrize("span", SPANS)
def test_span_resolves_in_newest_pmc(bench, span):
    from merlin import _native as nat

    names = {**bench.PMC_ALIAS, **bench.h3_gemm_names(nat)}.get(span, span)
    names = names if isinstance(names, tuple) else (names,)
    tag = newest_tag()
    pmc = os.path.join(REPO, "profiles", f"{tag}_pmc.json")
    assert os.path.exists(pmc), f"no PMC passes for the newest kernel trace {tag}"
    dd = json.load(open(pmc))
    trace = open(os.path.join(REPO, "profiles", f"{tag}_kernel_stats.csv")).read()
    # the span's first kernel ran in the newest trace and was counted in its PMC passes
    first = names[0]
    hit = [k for k in dd if k == first or k.startswith(first[:-1] + ",")] if first.endswith(">") else \
        [k for k in dd if k == first]
    assert len(hit) == 1, (span, first)
    assert f"\n{hit[0]}," in trace or f'\n"{hit[0]}",' in trace, (span, hit[0])
    assert bench.pmc_traffic(span) == sum(int(dd[k]["hbm_bytes_per_launch"]) for k in
                                          [hit[0]] + [n for n in names[1:] if n in dd])


def test_stale_pmc_passes_are_ignored(bench):
    """A PMC file older than the newest kernel trace is never read, even for a kernel only it holds."""
    tag = newest_tag()
    older = [f for f in glob.glob(os.path.join(REPO, "profiles", "*_pmc.json"))
             if os.path.basename(f).split("_")[0] < tag]
    only_old = set()
    for f in older:
        only_old |= set(json.load(open(f)))
    only_old -= set(json.load(open(os.path.join(REPO, "profiles", f"{tag}_pmc.json"))))
    from merlin import _native as nat

    aliases = {**bench.PMC_ALIAS, **bench.h3_gemm_names(nat)}
    only_old = sorted(k for k in only_old if "<" not in k and k.startswith("k_") and k not in aliases)
    assert only_old, "expected a kernel measured only by an older pass"
    assert bench.pmc_traffic(only_old[0]) is None


def test_env_tier_traffic_is_the_algorithmic_bytes(bench):
    """The 2M-env tier's k_env_step (bench.py env_large_tier, scripts/r06/gpu_envpmc.sh) moves its 168 algorithmic
    bytes per env-step and little more: PMC HBM bytes per launch within 5 % of 168 x 2^21."""
    from merlin.envs import ENV_STEP_BYTES

    t = bench.pmc_traffic("k_env_step_large")
    assert t is not None
    assert abs(t / (ENV_STEP_BYTES * (1 << 21)) - 1) < 0.05, t
