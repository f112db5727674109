"""How fast HBM state reaches a /dev/shm file and comes back: the copies behind the runner's rescue
snapshots (devspace_amd/rescue.py `_write`, `load`) when they are not staged in HBM.

Three ways, each for one write (device -> shared memory) and one read (shared memory -> device)
of --gib GiB, best of --reps:
  pageable    copy_ between the device tensor and a tensor over the file's mapping (the HIP
              runtime bounces pageable memory through its own small staging buffers);
  registered  the mapping is page-locked with hipHostRegister first, so the copy is one DMA
              straight into (out of) the shared-memory pages; the time includes the register and
              unregister calls;
  bounce      two pinned 64 MiB buffers: a DMA into one while the CPU copies the other to (from)
              the mapping.
Prints one JSON line.

    python scripts/shm_copy_cost.py [--gib 2] [--reps 3]
"""

import argparse
import json
import mmap
import os
import time

import torch

CH = 64 << 20


def _map(path, n, write):
    fresh = write and not (write == "recycled" and os.path.exists(path))
    f = open(path, "w+b" if fresh else "r+b")
    if fresh:
        os.posix_fallocate(f.fileno(), 0, n)
    return f, mmap.mmap(f.fileno(), n)


def write_pageable(src, path, write=True):
    f, mm = _map(path, src.numel(), write)
    buf = torch.frombuffer(mm, dtype=torch.uint8)
    buf.copy_(src)
    del buf
    mm.close()
    f.close()


def write_registered(src, path):
    n = src.numel()
    f, mm = _map(path, n, True)
    buf = torch.frombuffer(mm, dtype=torch.uint8)
    rt = torch.cuda.cudart()
    err = rt.cudaHostRegister(buf.data_ptr(), n, 0)
    if int(err) != 0:
        raise RuntimeError(f"hipHostRegister: {err}")
    try:
        buf.copy_(src, non_blocking=True)
        torch.cuda.current_stream().synchronize()
    finally:
        rt.cudaHostUnregister(buf.data_ptr())
    del buf
    mm.close()
    f.close()


def write_bounce(src, path, pins, stream, write=True):
    n = src.numel()
    f, mm = _map(path, n, write)
    buf = torch.frombuffer(mm, dtype=torch.uint8)
    ev = [torch.cuda.Event(), torch.cuda.Event()]
    chunks = [(o, min(CH, n - o)) for o in range(0, n, CH)]
    stream.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(stream):
        for i, (o, k) in enumerate(chunks[:2]):
            pins[i][:k].copy_(src[o:o + k], non_blocking=True)
            ev[i].record(stream)
        for i, (o, k) in enumerate(chunks):
            ev[i % 2].synchronize()
            buf[o:o + k].copy_(pins[i % 2][:k])
            if i + 2 < len(chunks):
                o2, k2 = chunks[i + 2]
                pins[i % 2][:k2].copy_(src[o2:o2 + k2], non_blocking=True)
                ev[i % 2].record(stream)
    del buf
    mm.close()
    f.close()


def read_pageable(path, n, dev):
    f = open(path, "rb")
    mm = mmap.mmap(f.fileno(), n, access=mmap.ACCESS_COPY)
    buf = torch.frombuffer(mm, dtype=torch.uint8)
    out = buf.to(dev)
    torch.cuda.synchronize()
    del buf
    mm.close()
    f.close()
    return out


def read_registered(path, n, dev):
    f, mm = _map(path, n, False)
    buf = torch.frombuffer(mm, dtype=torch.uint8)
    rt = torch.cuda.cudart()
    err = rt.cudaHostRegister(buf.data_ptr(), n, 0)
    if int(err) != 0:
        raise RuntimeError(f"hipHostRegister: {err}")
    try:
        out = torch.empty(n, dtype=torch.uint8, device=dev)
        out.copy_(buf, non_blocking=True)
        torch.cuda.current_stream().synchronize()
    finally:
        rt.cudaHostUnregister(buf.data_ptr())
    del buf
    mm.close()
    f.close()
    return out


def read_bounce(path, n, dev, pins, stream):
    f = open(path, "rb")
    mm = mmap.mmap(f.fileno(), n, access=mmap.ACCESS_COPY)
    buf = torch.frombuffer(mm, dtype=torch.uint8)
    out = torch.empty(n, dtype=torch.uint8, device=dev)
    ev = [torch.cuda.Event(), torch.cuda.Event()]
    chunks = [(o, min(CH, n - o)) for o in range(0, n, CH)]
    with torch.cuda.stream(stream):
        for i, (o, k) in enumerate(chunks):
            if i >= 2:
                ev[i % 2].synchronize()  # the DMA out of this buffer is done
            pins[i % 2][:k].copy_(buf[o:o + k])
            out[o:o + k].copy_(pins[i % 2][:k], non_blocking=True)
            ev[i % 2].record(stream)
    stream.synchronize()
    del buf
    mm.close()
    f.close()
    return out


def fallocate(path, n):
    if os.path.exists(path):
        os.unlink(path)
    with open(path, "w+b") as f:
        os.posix_fallocate(f.fileno(), 0, n)


def best(fn, reps):
    ts = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) * 1000.0)
    return round(min(ts), 1), [round(t, 1) for t in ts]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=float, default=2.0)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    n = int(args.gib * (1 << 30)) // CH * CH
    src = torch.randint(0, 255, (n,), dtype=torch.uint8, device=dev)
    path = f"/dev/shm/shm-copy-cost-{os.getpid()}.bin"
    pins = [torch.empty(CH, dtype=torch.uint8).pin_memory() for _ in range(2)]
    stream = torch.cuda.Stream(device=dev)
    out = {"what": "device <-> /dev/shm file copies of the rescue snapshot path", "gib": n / (1 << 30),
           "device": torch.cuda.get_device_name(0), "write_ms": {}, "read_ms": {}, "gbps": {}}
    try:
        for name, fn in (("pageable", lambda: write_pageable(src, path)),
                         ("registered", lambda: write_registered(src, path)),
                         ("fallocate_only", lambda: fallocate(path, n)),
                         ("pageable_recycled", lambda: write_pageable(src, path, "recycled")),
                         ("bounce_recycled", lambda: write_bounce(src, path, pins, stream, "recycled")),
                         ("bounce", lambda: write_bounce(src, path, pins, stream))):
            try:
                out["write_ms"][name] = best(fn, args.reps)
                out["gbps"]["write_" + name] = round(n / out["write_ms"][name][0] / 1e6, 2)
                if name == "fallocate_only":
                    continue
                with open(path, "rb") as f:  # what landed is what was on the device
                    mm = mmap.mmap(f.fileno(), n, access=mmap.ACCESS_READ)
                    head = torch.frombuffer(bytearray(mm[:1 << 20]), dtype=torch.uint8)
                    tail = torch.frombuffer(bytearray(mm[n - (1 << 20):]), dtype=torch.uint8)
                    mm.close()
                ok = torch.equal(head, src[:1 << 20].cpu()) and torch.equal(tail, src[n - (1 << 20):].cpu())
                out.setdefault("write_ok", {})[name] = bool(ok)
            except Exception as e:
                out["write_ms"][name] = f"{type(e).__name__}: {e}"
            if name in ("pageable", "registered", "bounce_recycled") and os.path.exists(path):
                os.unlink(path)
        for name, fn in (("pageable", lambda: read_pageable(path, n, dev)),
                         ("registered", lambda: read_registered(path, n, dev)),
                         ("bounce", lambda: read_bounce(path, n, dev, pins, stream))):
            try:
                res = {}
                out["read_ms"][name] = best(lambda: res.__setitem__("t", fn()), args.reps)
                out["gbps"]["read_" + name] = round(n / out["read_ms"][name][0] / 1e6, 2)
                out.setdefault("read_ok", {})[name] = bool(torch.equal(res["t"], src))
                del res
            except Exception as e:
                out["read_ms"][name] = f"{type(e).__name__}: {e}"
    finally:
        if os.path.exists(path):
            os.unlink(path)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
