"""Pre-tuned GEMM solutions for the update's fc1 GEMMs on gfx950 (PyTorch TunableOp).

hipBLASLt's heuristic pick for the update's fc1 shapes runs at ~110-120 TFLOP/s of the 157.3
fp32 MFMA peak.  An exhaustive search over the hipBLASLt and rocBLAS solutions
(scripts/tune_gemms.py, offline on an MI355X) finds faster kernels in its timing loop for all
three fc1 GEMMs and the window GEMMs, but inside the update most did not hold up: the searched
forward and split-K weight-gradient solutions measured 6-20 % slower there than hipBLASLt's own
pick (profiles/r02_tuning_ab.md), and with the searched input-gradient solution (a rocBLAS
global-split kernel, 965-1,020 -> 908 us per minibatch) -- together with the searched window
GEMMs, or alone -- the training loop turned non-finite after 10-38 iterations while every
checked call (each tuned GEMM re-run on the default path and compared, which serialises the
stream) agreed to 5e-7 and the same loop without them ran 60 iterations clean
(scripts/debug_nan.py).  So only the rollout's fixed-shape conv3 / fc1 GEMMs ship (rocBLAS
solutions, 62 -> 44 us and 40 -> 38 us per step, clean over 45+ iterations), as a TunableOp CSV
(tuning/gemm_gfx950.csv).  The machinery below (row / window padding to tuned counts, tuned
window GEMMs) stays for shapes a future file may hold.

The file is read once with tuning OFF, and TunableOp dispatch is switched on only around the
GEMMs it was made for (`with tuned(which):`); there a shape found in the file runs the recorded
solution, any other runs PyTorch's default, and every other GEMM of the process takes PyTorch's
usual path.  Nothing is timed or written at run time.  The file's validator lines (PyTorch /
HIP / hipBLASLt / rocBLAS versions, gfx950) make TunableOp reject it on any other stack.
MERLIN_GEMM_TUNING=0 switches it off; MERLIN_UNTUNED=rollout,dgrad,window switches groups off.
The file is loaded lazily, by the first GEMM that asks for it (`tuned()` / `padded_*`): the default
training path (h3 fc1 and window GEMMs, all-windows acting table) never does, so TunableOp stays off there."""
from __future__ import annotations

import contextlib
import os
import re

import torch

TUNED_FILE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tuning", "gemm_gfx950.csv")
ROW_BUCKET = 2048
WINDOW_BUCKET = 256  # the window GEMMs' row count (distinct windows of an update) is padded to this
_state = {"on": False, "tried": False, "rows": (), "windows": ()}


def enable(path: str = TUNED_FILE) -> bool:
    """Load the tuned solutions (once per process); True when they are in use."""
    if _state["tried"]:
        return _state["on"]
    _state["tried"] = True
    if os.environ.get("MERLIN_GEMM_TUNING", "1") == "0" or not torch.cuda.is_available() or not os.path.exists(path):
        return False
    if not torch.cuda.get_device_properties(torch.cuda.current_device()).gcnArchName.startswith("gfx950"):
        return False
    import torch.cuda.tunable as tunable

    tunable.tuning_enable(False)
    tunable.set_filename(path)
    _state["on"] = bool(tunable.read_file(path))
    tunable.enable(False)  # dispatch only inside tuned()
    if _state["on"]:
        text = open(path).read()
        _state["rows"] = tuple(sorted({int(m.group(1)) for m in re.finditer(r"nn_576_(\d+)_512_B_2", text)}))
        _state["windows"] = tuple(sorted({int(m.group(1)) for m in re.finditer(r"nn_576_(\d+)_64_B_2", text)}))
    return _state["on"]


@contextlib.contextmanager
def tuned(which: str = ""):
    """TunableOp dispatch (recorded solutions, no tuning) for the GEMMs inside the block."""
    if not _state["tried"] and torch.cuda.is_available():
        enable()
    if (not _state["on"] or (which and which in os.environ.get("MERLIN_UNTUNED", "").split(","))
            or os.environ.get("MERLIN_PAD_ONLY")):  # (testing: the padding without the tuned dispatch)
        yield
        return
    import torch.cuda.tunable as tunable

    tunable.enable(True)
    try:
        yield
    finally:
        tunable.enable(False)


def active() -> bool:
    return _state["on"]


def padded_windows(n: int) -> int:
    """The tuned window-GEMM row count to pad n windows to (n when none lies within WINDOW_BUCKET)."""
    if "window" in os.environ.get("MERLIN_UNTUNED", "").split(","):
        return n
    if not _state["tried"] and torch.cuda.is_available():
        enable()
    for r in _state["windows"]:
        if n <= r < n + WINDOW_BUCKET:
            return r
    return n


def padded_rows(n: int) -> int:
    """The tuned fc1 row count to pad n frames to (n itself when none lies within ROW_BUCKET)."""
    if "dgrad" in os.environ.get("MERLIN_UNTUNED", "").split(","):
        return n
    if not _state["tried"] and torch.cuda.is_available():
        enable()
    for r in _state["rows"]:  # (row counts of the dgrad entries: nn_576_<rows>_512)
        if n <= r < n + ROW_BUCKET:
            return r
    return n
