"""TEST INFRASTRUCTURE ONLY -- literal, object-level Python restatement of the
minigrid 3.0.0 semantics the MERLIN envs use, for small cases.

It exists to cross-check the C oracle (oracle/merlin_oracle.c), which uses
closed forms (view rotation) and its own PCG64/SeedSequence code.  This file
instead follows minigrid's code structure step by step (Grid.slice,
rotate_left applied dir+1 times, process_vis with its two passes, place_obj
rejection loop) and draws from numpy's real ``np.random.default_rng(seed)``
(== gymnasium ``seeding.np_random``: Generator(PCG64(SeedSequence(seed)))).

minigrid/gymnasium are not installed in this container, so the
minigrid-level semantics here are a restatement from the pinned public source
(minigrid 3.0.0, uv.lock:467-469): "parity unpinned" w.r.t. minigrid itself.
The MERLIN generator logic follows the reference files cited per function.
Only tests/ may import this module.
"""
from __future__ import annotations

import math
from collections import deque

import numpy as np

EMPTY, WALL, GOAL = None, "wall", "goal"
DIR_TO_VEC = [(1, 0), (0, 1), (-1, 0), (0, -1)]


class Grid:
    """minigrid core/grid.py Grid: flat list, index j*width+i."""

    def __init__(self, width, height):
        self.width, self.height = width, height
        self.grid = [None] * (width * height)

    def get(self, i, j):
        return self.grid[j * self.width + i]

    def set(self, i, j, v):
        self.grid[j * self.width + i] = v

    def wall_rect(self, x, y, w, h):
        for i in range(x, x + w):
            self.set(i, y, WALL)
            self.set(i, y + h - 1, WALL)
        for j in range(y, y + h):
            self.set(x, j, WALL)
            self.set(x + w - 1, j, WALL)

    def slice(self, topX, topY, width, height):
        g = Grid(width, height)
        for j in range(height):
            for i in range(width):
                x, y = topX + i, topY + j
                if 0 <= x < self.width and 0 <= y < self.height:
                    v = self.get(x, y)
                else:
                    v = WALL
                g.set(i, j, v)
        return g

    def rotate_left(self):
        g = Grid(self.height, self.width)
        for i in range(self.width):
            for j in range(self.height):
                g.set(j, g.height - 1 - i, self.get(i, j))
        return g

    def process_vis(self, agent_pos):
        mask = np.zeros((self.width, self.height), dtype=bool)
        mask[agent_pos[0], agent_pos[1]] = True
        for j in reversed(range(0, self.height)):
            for i in range(0, self.width - 1):
                if not mask[i, j]:
                    continue
                cell = self.get(i, j)
                if cell == WALL:  # cell and not cell.see_behind()
                    continue
                mask[i + 1, j] = True
                if j > 0:
                    mask[i + 1, j - 1] = True
                    mask[i, j - 1] = True
            for i in reversed(range(1, self.width)):
                if not mask[i, j]:
                    continue
                cell = self.get(i, j)
                if cell == WALL:
                    continue
                mask[i - 1, j] = True
                if j > 0:
                    mask[i - 1, j - 1] = True
                    mask[i, j - 1] = True
        for j in range(self.height):
            for i in range(self.width):
                if not mask[i, j]:
                    self.set(i, j, None)
        return mask


class LiteralEnv:
    """MiniGridEnv subset + MERLIN generators (src/custom_envs/*)."""

    def __init__(self, size=16, difficulty="mediumhard", max_steps=None):
        self.width = self.height = size
        self.difficulty = difficulty
        self.max_steps = 4 * size * size if max_steps is None else max_steps  # base_env.py:32-33
        self.agent_view_size = 7
        self.np_random = None

    # --- minigrid_env.py helpers ---
    def _rand_int(self, lo, hi):
        return int(self.np_random.integers(lo, hi))

    def place_obj(self, obj, top=None, size=None, max_tries=math.inf):
        top = (0, 0) if top is None else (max(top[0], 0), max(top[1], 0))
        if size is None:
            size = (self.grid.width, self.grid.height)
        num_tries = 0
        while True:
            if num_tries > max_tries:
                raise RecursionError("rejection sampling failed in place_obj")
            num_tries += 1
            pos = (
                self._rand_int(top[0], min(top[0] + size[0], self.grid.width)),
                self._rand_int(top[1], min(top[1] + size[1], self.grid.height)),
            )
            if self.grid.get(*pos) is not None:
                continue
            if tuple(pos) == tuple(self.agent_pos):
                continue
            break
        self.grid.set(pos[0], pos[1], obj)
        return pos

    def place_agent(self, top=None, size=None):
        self.agent_pos = (-1, -1)
        pos = self.place_obj(None, top, size)
        self.agent_pos = pos
        self.agent_dir = self._rand_int(0, 4)
        return pos

    # --- generators ---
    def _reachable(self, s, g):  # medium_hard_env.py:47-74
        visited = {s}
        q = deque([s])
        while q:
            cx, cy = q.popleft()
            if (cx, cy) == g:
                return True
            for dx, dy in [(0, 1), (1, 0), (0, -1), (-1, 0)]:
                nx, ny = cx + dx, cy + dy
                if 0 <= nx < self.width and 0 <= ny < self.height and (nx, ny) not in visited:
                    c = self.grid.get(nx, ny)
                    if c is None or c == GOAL or (nx, ny) == g:
                        visited.add((nx, ny))
                        q.append((nx, ny))
        return False

    def _fallback(self):
        self.grid = Grid(self.width, self.height)
        self.grid.wall_rect(0, 0, self.width, self.height)
        self.place_agent()
        self.goal_pos = self.place_obj(GOAL)

    def _gen_grid(self):
        W, H = self.width, self.height
        d = self.difficulty
        if d == "easy":  # easy_env.py:19-39
            self.grid = Grid(W, H)
            self.grid.wall_rect(0, 0, W, H)
            self.place_agent()
            self.grid.set(W - 5, H - 5, GOAL)
            self.goal_pos = (W - 5, H - 5)
            return
        if d == "medium":  # medium_env.py:19-33
            self.grid = Grid(W, H)
            self.grid.wall_rect(0, 0, W, H)
            self.place_agent()
            self.goal_pos = self.place_obj(GOAL)
            return
        for _ in range(100):
            self.grid = Grid(W, H)
            self.grid.wall_rect(0, 0, W, H)
            if d == "mediumhard":  # medium_hard_env.py:12-38
                playable = (W - 2) * (H - 2)
                n = self._rand_int(max(1, int(playable * 0.10)), max(1, int(playable * 0.20)) + 1)
                for _ in range(n):
                    self.place_obj(WALL, max_tries=100)
                self.place_agent()
                self.goal_pos = self.place_obj(GOAL)
            elif d == "hard":  # hard_env.py:11-66
                mid = W // 2
                large = W > 10
                num_gaps = self._rand_int(2, 6) if large else 1
                gaps = self.np_random.choice(list(range(1, H - 1)), size=num_gaps, replace=False)
                for i in range(H):
                    if i == 0 or i == H - 1:
                        continue
                    if i not in gaps:
                        self.grid.set(mid, i, WALL)
                if large:
                    for _ in range(self._rand_int(6, 13)):
                        for _ in range(10):
                            x = self._rand_int(1, W - 1)
                            y = self._rand_int(1, H - 1)
                            if x != mid and self.grid.get(x, y) is None:
                                self.grid.set(x, y, WALL)
                                break
                self.goal_pos = self.place_obj(GOAL, top=(mid + 1, 0), size=(W - mid - 1, H))
                self.place_agent(top=(1, 1), size=(mid - 1, H - 2))
            else:  # hardest_env.py:20-64
                mx, my = W // 2, H // 2
                for y in range(1, H - 1):
                    self.grid.set(mx, y, WALL)
                for x in range(1, W - 1):
                    self.grid.set(x, my, WALL)
                self.grid.set(mx, self._rand_int(2, my - 1), None)
                self.grid.set(mx, self._rand_int(my + 1, H - 2), None)
                self.grid.set(self._rand_int(2, mx - 1), my, None)
                self.grid.set(self._rand_int(mx + 1, W - 2), my, None)
                for _ in range(self._rand_int(6, 13)):
                    x = self._rand_int(1, W - 1)
                    y = self._rand_int(1, H - 1)
                    if self.grid.get(x, y) is None and x != mx and y != my:
                        self.grid.set(x, y, WALL)
                self.place_agent()
                self.goal_pos = self.place_obj(GOAL)
            if self._reachable(tuple(self.agent_pos), tuple(self.goal_pos)):
                return
        self._fallback()

    # --- gym API ---
    def reset(self, seed=None):
        if seed is not None:
            self.np_random = np.random.default_rng(seed)
        self.agent_pos = (-1, -1)
        self.agent_dir = -1
        self._gen_grid()
        self.step_count = 0
        return self.view_codes()

    def step(self, action):
        self.step_count += 1
        reward, terminated, truncated = 0, False, False
        fx = self.agent_pos[0] + DIR_TO_VEC[self.agent_dir][0]
        fy = self.agent_pos[1] + DIR_TO_VEC[self.agent_dir][1]
        fwd = self.grid.get(fx, fy)
        if action == 0:
            self.agent_dir -= 1
            if self.agent_dir < 0:
                self.agent_dir += 4
        elif action == 1:
            self.agent_dir = (self.agent_dir + 1) % 4
        elif action == 2:
            if fwd is None or fwd == GOAL:
                self.agent_pos = (fx, fy)
            if fwd == GOAL:
                terminated = True
                reward = 1 - 0.9 * (self.step_count / self.max_steps)
        else:
            raise ValueError(action)
        if self.step_count >= self.max_steps:
            truncated = True
        return self.view_codes(), reward, terminated, truncated

    def view_codes(self):
        """gen_obs_grid + get_pov_render tile selection -> 7x7 codes [vj][vi]."""
        v = self.agent_view_size
        ax, ay = self.agent_pos
        d = self.agent_dir
        if d == 0:
            tx, ty = ax, ay - v // 2
        elif d == 1:
            tx, ty = ax - v // 2, ay
        elif d == 2:
            tx, ty = ax - v + 1, ay - v // 2
        else:
            tx, ty = ax - v // 2, ay - v + 1
        g = self.grid.slice(tx, ty, v, v)
        for _ in range(d + 1):
            g = g.rotate_left()
        mask = g.process_vis(agent_pos=(v // 2, v - 1))
        g.set(v // 2, v - 1, None)
        codes = np.zeros((v, v), dtype=np.uint8)
        for j in range(v):
            for i in range(v):
                if (i, j) == (v // 2, v - 1):
                    c = 4
                elif not mask[i, j]:
                    c = 0
                else:
                    cell = g.get(i, j)
                    c = 2 if cell == WALL else 3 if cell == GOAL else 1
                codes[j, i] = c
        return codes

    def cells(self):
        out = np.zeros((self.height, self.width), dtype=np.uint8)
        for j in range(self.height):
            for i in range(self.width):
                c = self.grid.get(i, j)
                out[j, i] = 1 if c == WALL else 2 if c == GOAL else 0
        return out

    def full_obs(self):
        """FullyObsWrapper.observation (minigrid 3.0.0 wrappers.py) after ImgObsWrapper: Grid.encode() of the whole
        grid -- [i][j] = (OBJECT_TO_IDX, COLOR_TO_IDX, state) of cell (i, j), None as empty (1, 0, 0), Wall (2, grey
        5, 0), Goal (8, green 1, 0) -- with the agent's cell overwritten by (agent 10, red 0, agent_dir)."""
        out = np.zeros((self.width, self.height, 3), dtype=np.uint8)
        for i in range(self.width):
            for j in range(self.height):
                c = self.grid.get(i, j)
                out[i, j] = (2, 5, 0) if c == WALL else (8, 1, 0) if c == GOAL else (1, 0, 0)
        ax, ay = self.agent_pos
        out[ax, ay] = (10, 0, self.agent_dir)
        return out


def full_obs_from_state(walls, agent_pos, agent_dir, goal_pos, size):
    """The same observation from the bit-row state MerlinVecEnv.get_state reports (walls[y] bit x = wall at
    (x, y)): the checker of merlin_env_full_obs."""
    out = np.zeros((size, size, 3), dtype=np.uint8)
    out[...] = (1, 0, 0)
    for y in range(size):
        for x in range(size):
            if (int(walls[y]) >> x) & 1:
                out[x, y] = (2, 5, 0)
    out[int(goal_pos[0]), int(goal_pos[1])] = (8, 1, 0)
    out[int(agent_pos[0]), int(agent_pos[1])] = (10, 0, int(agent_dir))
    return out

