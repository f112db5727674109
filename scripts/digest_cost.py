"""What the rescue snapshots' content digest costs (devspace_amd/rescue.py `digests`): the gfx950
`state_digest` kernel (one HBM read of the state, one launch for all tensors) against the same
numbers computed with torch ops on the device and on the CPU, for a training state of a given
size. Prints one JSON line (scripts/gpu_tier.sh digest).

  python scripts/digest_cost.py [--gib 2] [--tensors 64] [--rounds 5]
"""

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from devspace_amd import rescue  # noqa: E402


def _time(fn, rounds, sync):
    out = []
    for _ in range(rounds):
        sync()
        t0 = time.perf_counter()
        fn()
        sync()
        out.append((time.perf_counter() - t0) * 1000.0)
    out.sort()
    return out[len(out) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=float, default=2.0)
    ap.add_argument("--tensors", type=int, default=64)
    ap.add_argument("--rounds", type=int, default=5)
    args = ap.parse_args()
    assert torch.cuda.is_available(), "needs a GPU"
    dev = torch.device("cuda", 0)
    total = int(args.gib * 2**30)
    per = total // args.tensors // 2  # bf16 elements per tensor
    torch.manual_seed(0)
    state = [torch.randn(per, device=dev, dtype=torch.bfloat16) for _ in range(args.tensors)]
    nbytes = sum(t.numel() * t.element_size() for t in state)
    kernel = rescue._digest_kernel()
    assert kernel is not None, "fused-ops extension with state_digest not loaded"
    sync = torch.cuda.synchronize
    words = [t.reshape(-1).view(torch.int64) for t in state]
    rescue.digests(state)  # warm-up (extension load, caches)
    k_ms = _time(lambda: kernel.state_digest(words), args.rounds, sync)
    full_ms = _time(lambda: rescue.digests(state), args.rounds, sync)
    torch_ms = _time(lambda: [rescue._digest_rows_torch(w) for w in words], max(1, args.rounds // 2), sync)
    assert torch.equal(kernel.state_digest(words[:2]).cpu(),
                       torch.cat([rescue._digest_rows_torch(w) for w in words[:2]]).cpu())
    cpu_words = [w[: (64 << 20) // 8].cpu() for w in words[:1]]  # 64 MiB on the CPU, scaled
    cpu_ms = _time(lambda: [rescue._digest_rows_torch(w) for w in cpu_words], 3, lambda: None) * (nbytes / (64 << 20))
    host = [w.cpu() for w in words]  # the same state in host memory: the extension's one-pass CPU path
    cpu_ext_ms = _time(lambda: kernel.state_digest_cpu(host), 3, lambda: None)
    print(json.dumps({
        "state_gib": round(nbytes / 2**30, 3), "tensors": args.tensors,
        "kernel_ms": round(k_ms, 3), "kernel_tb_s": round(nbytes / k_ms / 1e9, 2),
        "digests_ms": round(full_ms, 3),
        "torch_on_device_ms": round(torch_ms, 2), "torch_on_cpu_ms_est": round(cpu_ms, 1),
        "cpu_one_pass_ms": round(cpu_ext_ms, 1), "cpu_threads": torch.get_num_threads(),
        "kernel_speedup_vs_torch_on_device": round(torch_ms / k_ms, 1),
        "what": "rescue.digests of a bf16 training state: (sum, position-keyed mixed sum) per 64 Ki-word row; "
                "kernel = one state_digest launch; digests = kernel + one host copy + BLAKE2b per tensor",
        "device": torch.cuda.get_device_name(0),
    }))


if __name__ == "__main__":
    main()
