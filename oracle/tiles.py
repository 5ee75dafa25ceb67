"""TEST INFRASTRUCTURE ONLY -- numpy restatement of minigrid 3.0.0's tile
renderer (minigrid/core/grid.py Grid.render_tile, minigrid/utils/rendering.py
fill_coords / point_in_rect / point_in_triangle / rotate_fn / highlight_img /
downsample), with numpy dtypes kept as in that code (float32 triangle vertices,
float64 sample points, uint8 image, float64 mean in downsample, truncating
cast when the tile is written into the uint8 frame in Grid.render).

Produces the 5 tiles that can appear in RGBImgPartialObsWrapper(tile_size=8)
observations of the MERLIN envs (only Wall/Goal/empty cells, agent always at
view (3,6) facing up, highlight = vis mask):
    0 dark empty (not visible) | 1 lit empty | 2 lit wall | 3 lit goal | 4 agent
Parity: minigrid is absent here -> restatement, pinned only by the R-channel
values the survey recorded.  Only tests/ and the
golden-generation script import this module.
"""
from __future__ import annotations

import math

import numpy as np

GREY = (100, 100, 100)  # COLORS["grey"]
GREEN = (0, 255, 0)  # COLORS["green"]
RED = (255, 0, 0)


def point_in_rect(xmin, xmax, ymin, ymax):
    def fn(x, y):
        return x >= xmin and x <= xmax and y >= ymin and y <= ymax

    return fn


def point_in_triangle(a, b, c):
    a = np.array(a, dtype=np.float32)
    b = np.array(b, dtype=np.float32)
    c = np.array(c, dtype=np.float32)

    def fn(x, y):
        v0 = c - a
        v1 = b - a
        v2 = np.array((x, y)) - a
        dot00 = np.dot(v0, v0)
        dot01 = np.dot(v0, v1)
        dot02 = np.dot(v0, v2)
        dot11 = np.dot(v1, v1)
        dot12 = np.dot(v1, v2)
        inv_denom = 1 / (dot00 * dot11 - dot01 * dot01)
        u = (dot11 * dot02 - dot01 * dot12) * inv_denom
        v = (dot00 * dot12 - dot01 * dot02) * inv_denom
        return (u >= 0) and (v >= 0) and (u + v) < 1

    return fn


def rotate_fn(fin, cx, cy, theta):
    def fout(x, y):
        x = x - cx
        y = y - cy
        x2 = cx + x * math.cos(-theta) - y * math.sin(-theta)
        y2 = cy + y * math.cos(-theta) + x * math.sin(-theta)
        return fin(x2, y2)

    return fout


def fill_coords(img, fn, color):
    for y in range(img.shape[0]):
        for x in range(img.shape[1]):
            yf = (y + 0.5) / img.shape[0]
            xf = (x + 0.5) / img.shape[1]
            if fn(xf, yf):
                img[y, x] = color
    return img


def highlight_img(img, color=(255, 255, 255), alpha=0.30):
    blend_img = img + alpha * (np.array(color, dtype=np.uint8) - img)
    blend_img = blend_img.clip(0, 255).astype(np.uint8)
    img[:, :, :] = blend_img


def downsample(img, factor):
    img = img.reshape([img.shape[0] // factor, factor, img.shape[1] // factor, factor, 3])
    img = img.mean(axis=3)
    img = img.mean(axis=1)
    return img


def render_tile(obj, agent_dir=None, highlight=False, tile_size=8, subdivs=3):
    img = np.zeros((tile_size * subdivs, tile_size * subdivs, 3), dtype=np.uint8)
    fill_coords(img, point_in_rect(0, 0.031, 0, 1), GREY)
    fill_coords(img, point_in_rect(0, 1, 0, 0.031), GREY)
    if obj == "wall":
        fill_coords(img, point_in_rect(0, 1, 0, 1), GREY)
    elif obj == "goal":
        fill_coords(img, point_in_rect(0, 1, 0, 1), GREEN)
    if agent_dir is not None:
        tri = point_in_triangle((0.12, 0.19), (0.87, 0.50), (0.12, 0.81))
        tri = rotate_fn(tri, cx=0.5, cy=0.5, theta=0.5 * math.pi * agent_dir)
        fill_coords(img, tri, RED)
    if highlight:
        highlight_img(img)
    img = downsample(img, subdivs)
    # Grid.render: img[ymin:ymax, xmin:xmax, :] = tile_img (float64 -> uint8)
    out = np.zeros((tile_size, tile_size, 3), dtype=np.uint8)
    out[:, :, :] = img
    return out


def build_atlas(tile_size=8):
    """uint8[5, ts, ts, 3] in class order (dark, lit empty, lit wall, lit goal, agent)."""
    return np.stack(
        [
            render_tile(None, None, False, tile_size),
            render_tile(None, None, True, tile_size),
            render_tile("wall", None, True, tile_size),
            render_tile("goal", None, True, tile_size),
            render_tile(None, 3, True, tile_size),
        ]
    )


if __name__ == "__main__":
    a = build_atlas()
    for k in range(5):
        print(k, a[k, :, :, 0].tolist())
