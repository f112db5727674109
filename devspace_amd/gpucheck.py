"""In-pod GPU check used by `devspace analyze` for MI355X pods.

Kubernetes only knows that `amd.com/gpu: N` was scheduled; this reports what the container
can actually use: device nodes (/dev/kfd, /dev/dri), visible devices, and for each device a
measured MFMA self-test, HBM3E copy bandwidth and bf16 MFMA throughput (HIP kernels in
devspace_amd/ops/gpuprobe.hip), compared against MI355X expectations.

    python -m devspace_amd.gpucheck [--quick] [--json]
"""

from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys

# MI355X reference figures (MI355X_MICROARCH.md: 8 TB/s HBM spec, ~6.3 TB/s achievable float4
# copy; ~2.5 PF dense bf16 spec).
HBM_EXPECTED_GBPS = 6300.0
BF16_PEAK_TFLOPS = 2500.0
HBM_BYTES_PER_GPU = 288 * 10**9


class Probe:
    def __init__(self, path=None):
        from devspace_amd.ops import build as ops_build

        path = path or ops_build.lib_path()
        if not os.path.exists(path):
            ops_build.build_probe()
        self.lib = ctypes.CDLL(path)
        self.lib.gp_device_count.restype = ctypes.c_int
        self.lib.gp_device_info.argtypes = [ctypes.c_int, ctypes.c_char_p, ctypes.c_int]
        self.lib.gp_device_info.restype = ctypes.c_int
        self.lib.gp_mfma_selftest.argtypes = [ctypes.c_int]
        self.lib.gp_mfma_selftest.restype = ctypes.c_double
        self.lib.gp_hbm_copy_gbps.argtypes = [ctypes.c_int, ctypes.c_size_t, ctypes.c_int]
        self.lib.gp_hbm_copy_gbps.restype = ctypes.c_double
        self.lib.gp_hbm_copy_gbps_cfg.argtypes = [ctypes.c_int, ctypes.c_size_t, ctypes.c_int, ctypes.c_int,
                                                  ctypes.c_int, ctypes.c_int]
        self.lib.gp_hbm_copy_gbps_cfg.restype = ctypes.c_double
        self.lib.gp_mfma_bf16_tflops.argtypes = [ctypes.c_int, ctypes.c_int]
        self.lib.gp_mfma_bf16_tflops.restype = ctypes.c_double
        self.lib.gp_last_error.restype = ctypes.c_char_p
        self.lib.gp_peer_access.argtypes = [ctypes.c_int, ctypes.c_int]
        self.lib.gp_peer_access.restype = ctypes.c_int
        self.lib.gp_peer_copy_gbps.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_size_t, ctypes.c_int]
        self.lib.gp_peer_copy_gbps.restype = ctypes.c_double

    def count(self):
        return self.lib.gp_device_count()

    def info(self, dev):
        buf = ctypes.create_string_buffer(2048)
        if self.lib.gp_device_info(dev, buf, len(buf)) != 0:
            raise RuntimeError(self.lib.gp_last_error().decode())
        return json.loads(buf.value.decode())

    def selftest(self, dev):
        return self.lib.gp_mfma_selftest(dev)

    def hbm_gbps(self, dev, nbytes=1 << 30, iters=10):
        return self.lib.gp_hbm_copy_gbps(dev, nbytes, iters)

    def hbm_gbps_cfg(self, dev, unroll, nontemporal, blocks_per_cu, nbytes=1 << 30, iters=10):
        return self.lib.gp_hbm_copy_gbps_cfg(dev, nbytes, iters, unroll, int(nontemporal), blocks_per_cu)

    def mfma_tflops(self, dev, iters=20000):
        return self.lib.gp_mfma_bf16_tflops(dev, iters)

    def peer_access(self, a, b):
        return self.lib.gp_peer_access(a, b)

    def peer_gbps(self, a, b, nbytes=256 << 20, iters=4):
        return self.lib.gp_peer_copy_gbps(a, b, nbytes, iters)


def peer_check(probe, n, quick=False):
    """Every ordered device pair of the pod: peer access (xGMI) and copy bandwidth. RCCL's
    all-reduce over an 8-GPU ring is bound by its slowest link, so one pair without peer access
    or far below the others (a copy staged through the host, a degraded link) is reported.
    Returns (pairs, problems)."""
    pairs, problems = [], []
    for a in range(n):
        for b in range(n):
            if a == b:
                continue
            acc = probe.peer_access(a, b)
            gbps = probe.peer_gbps(a, b, nbytes=(64 << 20) if quick else (256 << 20), iters=2 if quick else 4)
            pairs.append({"src": a, "dst": b, "peer_access": acc == 1, "copy_gbps": round(gbps, 1)})
            if acc != 1:
                problems.append(f"gpu{a} -> gpu{b}: no peer access (RCCL falls back to copies through host memory)")
            elif gbps <= 0:
                problems.append(f"gpu{a} -> gpu{b}: peer copy failed")
    rates = sorted(p["copy_gbps"] for p in pairs if p["copy_gbps"] > 0)
    if rates:
        median = rates[len(rates) // 2]
        for p in pairs:
            if p["peer_access"] and 0 < p["copy_gbps"] < 0.5 * median:
                problems.append(f"gpu{p['src']} -> gpu{p['dst']}: peer copy {p['copy_gbps']:.0f} GB/s, under half the "
                                f"median pair ({median:.0f} GB/s): degraded link")
    return pairs, problems


def device_nodes():
    return {
        "/dev/kfd": os.path.exists("/dev/kfd"),
        "/dev/dri": os.path.isdir("/dev/dri"),
        "HIP_VISIBLE_DEVICES": os.environ.get("HIP_VISIBLE_DEVICES"),
        "ROCR_VISIBLE_DEVICES": os.environ.get("ROCR_VISIBLE_DEVICES"),
    }


def run(quick=False):
    report = {"nodes": device_nodes(), "devices": [], "problems": []}
    if not report["nodes"]["/dev/kfd"]:
        report["problems"].append("/dev/kfd missing: the pod did not get the AMD GPU device plugin's devices")
    try:
        probe = Probe()
    except OSError as e:
        report["problems"].append(f"cannot load HIP runtime / probe library: {e}")
        return report
    n = probe.count()
    if n == 0:
        report["problems"].append("no HIP devices visible (check amd.com/gpu request and HIP_VISIBLE_DEVICES)")
    for d in range(n):
        info = probe.info(d)
        err = probe.selftest(d)
        info["mfma_selftest_max_abs_err"] = err
        if err != 0.0:
            report["problems"].append(f"gpu{d}: MFMA self-test failed (max abs err {err})")
        if not quick:
            gbps = probe.hbm_gbps(d)
            tf = probe.mfma_tflops(d)
            info["hbm_copy_gbps"] = round(gbps, 1)
            info["hbm_copy_pct_of_achievable"] = round(100.0 * gbps / HBM_EXPECTED_GBPS, 1)
            info["mfma_bf16_tflops"] = round(tf, 1)
            info["mfma_bf16_pct_of_peak"] = round(100.0 * tf / BF16_PEAK_TFLOPS, 1)
            if "gfx950" in info.get("arch", "") and gbps < 0.5 * HBM_EXPECTED_GBPS:
                report["problems"].append(f"gpu{d}: HBM bandwidth {gbps:.0f} GB/s is below 50% of expected")
        report["devices"].append(info)
    if n > 1:  # `analyze --gpu-probe` runs --quick: a short peer pass (64 MiB per pair)
        report["peers"], probs = peer_check(probe, n, quick)
        report["problems"] += probs
    return report


def sweep_copy(dev=0, nbytes=1 << 30):
    """Copy-kernel configuration sweep (unroll x nontemporal x blocks/CU) -> list of rows."""
    probe = Probe()
    rows = []
    for unroll in (1, 2, 4, 8):
        for nt in (False, True):
            for bpc in (1, 2, 3, 4, 8, 16):
                gbps = probe.hbm_gbps_cfg(dev, unroll, nt, bpc, nbytes=nbytes)
                rows.append({"unroll": unroll, "nontemporal": nt, "blocks_per_cu": bpc, "gbps": round(gbps, 1)})
    return rows


def main(argv=None):
    ap = argparse.ArgumentParser(prog="devspace_amd.gpucheck")
    ap.add_argument("--quick", action="store_true", help="self-test only, no bandwidth/throughput runs")
    ap.add_argument("--json", action="store_true")
    ap.add_argument("--sweep-copy", action="store_true", help="HBM copy kernel tuning sweep on gpu0")
    args = ap.parse_args(argv)
    if args.sweep_copy:
        rows = sweep_copy()
        for r in sorted(rows, key=lambda r: -r["gbps"]):
            print(f"unroll={r['unroll']} nt={int(r['nontemporal'])} blocks/CU={r['blocks_per_cu']:>2} "
                  f"{r['gbps']:8.1f} GB/s ({100.0 * r['gbps'] / HBM_EXPECTED_GBPS:5.1f}% of achievable)")
        return 0
    rep = run(quick=args.quick)
    if args.json:
        print(json.dumps(rep))
    else:
        for dev in rep["devices"]:
            print(
                f"gpu{dev['index']}: {dev['name']} {dev['arch']} CUs={dev['compute_units']} "
                f"HBM={dev['hbm_total_bytes'] / 1e9:.0f}GB selftest_err={dev['mfma_selftest_max_abs_err']} "
                f"hbm={dev.get('hbm_copy_gbps')}GB/s mfma_bf16={dev.get('mfma_bf16_tflops')}TF/s"
            )
        peers = rep.get("peers") or []
        if peers:
            rates = sorted(p["copy_gbps"] for p in peers)
            print(f"peers: {sum(p['peer_access'] for p in peers)}/{len(peers)} pairs with peer access, copy "
                  f"{rates[0]:.0f}-{rates[-1]:.0f} GB/s (median {rates[len(rates) // 2]:.0f})")
        for p in rep["problems"]:
            print(f"problem: {p}")
    return 1 if rep["problems"] else 0


if __name__ == "__main__":
    sys.exit(main())
