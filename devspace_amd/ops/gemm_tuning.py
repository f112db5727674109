"""Pre-tuned hipBLASLt/rocBLAS GEMM solutions for MI355X (gfx950), via PyTorch TunableOp.

The library heuristics pick a GEMM kernel per shape from a generic table; on the skinny
token-count x hidden shapes of a dev-pod training step they leave throughput on the table.
TunableOp benchmarks every hipBLASLt/rocBLAS solution for a shape once and records the winner.
We ship the winners for the example workloads (`tuned/gemm_gfx950.csv`, produced on an MI355X
by `scripts/tune_gemms.py`) and load them read-only in every pod process, so the tuned kernels
are used from the first step with no tuning cost on the hot-reload path.

Modes (runner flag `--gemm-tuning` / env `DEVSPACE_GEMM_TUNING`):

    off      (default) library heuristics only
    shipped  use the shipped table when the device is gfx950; unknown shapes keep
             the heuristic choice, nothing is tuned or written
    online   like shipped, plus tune unseen shapes at first use and persist them to
             DEVSPACE_GEMM_TUNING_FILE (default ~/.cache/devspace/gemm_tuned.csv) so later
             process starts (and hot reloads, which keep the process) reuse them

Measured on MI355X for the rocm-pytorch TinyLM step (profiles/r1_gemm_tunableop_ab.json):
heuristic 3.755 ms vs tuned 3.749 ms, i.e. hipBLASLt's heuristic already picks the best
library kernel for those shapes — hence `off` by default; the modes pay off for user models
whose shapes the heuristic table covers badly.

TunableOp validates the file header (PyTorch, ROCm, hipBLASLt versions and the gfx arch): a
table from another stack is ignored by PyTorch itself, so a stale file can never pick a
wrong kernel.
"""

from __future__ import annotations

import os

SHIPPED = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tuned", "gemm_gfx950.csv")
MODES = ("off", "shipped", "online")


def _arch(device) -> str:
    import torch

    try:
        return torch.cuda.get_device_properties(device).gcnArchName.split(":")[0]
    except Exception:  # pragma: no cover - no GPU / no ROCm
        return ""


def apply(mode: str | None = None, device=None) -> dict:
    """Configure TunableOp for this process. Returns a small report for logging."""
    import torch

    mode = (mode or os.environ.get("DEVSPACE_GEMM_TUNING") or "off").lower()
    if mode not in MODES:
        raise ValueError(f"gemm tuning mode must be one of {MODES}, got {mode!r}")
    report = {"mode": mode, "active": False, "entries": 0}
    if mode == "off" or not torch.cuda.is_available() or torch.version.hip is None:
        return report
    arch = _arch(device if device is not None else torch.cuda.current_device())
    tunable = torch.cuda.tunable
    if mode == "shipped":
        if arch != "gfx950" or not os.path.exists(SHIPPED):
            return report
        # read-only: with tuning disabled TunableOp never writes its results file back
        tunable.enable(True)
        tunable.tuning_enable(False)
        tunable.record_untuned_enable(False)
        tunable.set_filename(SHIPPED)
        ok = tunable.read_file(SHIPPED)
        report.update(active=bool(ok), entries=_count(SHIPPED), file=SHIPPED)
        if not ok:
            tunable.enable(False)
        return report
    # online
    path = os.environ.get("DEVSPACE_GEMM_TUNING_FILE") or os.path.join(
        os.path.expanduser("~"), ".cache", "devspace", "gemm_tuned.csv")
    os.makedirs(os.path.dirname(path), exist_ok=True)
    tunable.enable(True)
    tunable.tuning_enable(True)
    tunable.set_max_tuning_duration(int(os.environ.get("DEVSPACE_GEMM_TUNING_MS", "30")))
    if arch == "gfx950" and os.path.exists(SHIPPED):
        tunable.read_file(SHIPPED)
    if os.path.exists(path):
        tunable.read_file(path)
    tunable.set_filename(path)
    report.update(active=True, entries=_count(path) + _count(SHIPPED), file=path)
    return report


def _count(path: str) -> int:
    try:
        with open(path) as f:
            return sum(1 for line in f if line.strip() and not line.startswith("Validator"))
    except OSError:
        return 0
