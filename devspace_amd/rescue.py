"""Rescue snapshots: training state that survives a restart of the runner's rank group
(devspace_amd/runner.py, devspace_amd/supervise.py).

The reference's restart-per-change model (nodemon in examples/quickstart/package.json:7, the
redeploy loop of cmd/dev.go:225-234) starts every process from nothing; a training run cannot
afford that, so the ranks snapshot their state into the pod's shared memory and a restarted group
resumes from it.
"""

from __future__ import annotations

import hashlib
import mmap
import os
import re
import threading
import time


def _close_mapping(mm) -> None:
    try:
        mm.close()
    except BufferError:  # a tensor view still alive (an exception's frame): the GC closes it
        pass


_CHUNK = 64 << 20  # bytes per pinned bounce buffer
_BOUNCE_MIN = 8 << 20  # device tensors at least this large are restored through the bounce buffers
_bounce = {"bufs": None, "lock": threading.Lock()}


def _pinned_pair():
    """Two page-locked 64 MiB host buffers, allocated once per process."""
    if _bounce["bufs"] is None:
        import torch

        _bounce["bufs"] = [torch.empty(_CHUNK, dtype=torch.uint8).pin_memory() for _ in range(2)]
    return _bounce["bufs"]


def _flat_bytes(t):
    import torch

    return t.reshape(-1).view(torch.uint8)


def _h2d(out, src) -> None:
    """The mapped shared memory `src` (uint8) -> the contiguous device tensor `out`: the CPU copies
    one 64 MiB chunk into a pinned buffer while the DMA of the other runs. A .to(device) of the
    pageable mapping goes through the HIP runtime's small staging buffers instead: 2 GiB took
    501-567 ms that way against 80-106 ms this way (profiles/r5_shm_copy.json), and a 2.5 GB
    TinyLM restore went from 760 ms to 113-141 ms (profiles/r5_rescue_restore_bounce.json)."""
    import torch

    d, n = _flat_bytes(out), src.numel()
    stream = torch.cuda.current_stream(out.device)
    # (the copies go to the current device's current stream: make that `out`'s, the events' one)
    with _bounce["lock"], torch.cuda.device(out.device):
        pins = _pinned_pair()
        evs = [torch.cuda.Event(), torch.cuda.Event()]
        for i, o in enumerate(range(0, n, _CHUNK)):
            k = min(_CHUNK, n - o)
            if i >= 2:
                evs[i % 2].synchronize()  # the DMA out of this buffer is done
            pins[i % 2][:k].copy_(src[o:o + k])
            d[o:o + k].copy_(pins[i % 2][:k], non_blocking=True)
            evs[i % 2].record(stream)
        for e in evs:  # the pair is free for the next copy
            e.synchronize()


class RescueSkipped(Exception):
    """A snapshot that cannot be taken this time (not enough shared memory) or ever (the state
    holds something that is not tensors, containers and scalars)."""


_ROW = 1 << 16  # int64 words per digest row
_GOLDEN, _MIX1, _MIX2 = (x - (1 << 64) for x in (0x9E3779B97F4A7C15, 0xBF58476D1CE4E5B9, 0x94D049BB133111EB))
_TORCH_ROWS = 8  # rows per chunk of the torch path: 4 MiB temporaries, reused (in place)


def _digest_rows_torch(v):
    """(S, M) per row of the int64 words `v`, as the gfx950 kernel `state_digest` computes them
    (devspace_amd/ops/fused_ops.hip): S = sum w_i, M = sum mix(w_i ^ (i + 1) * golden) mod 2^64
    with mix the splitmix64 finalizer. Integer arithmetic wraps, so both paths agree bit for bit.
    In-place ops on two reused chunk buffers: about 4 GB/s on 8 CPU threads (a fresh tensor per
    op ran at a quarter of that)."""
    import torch

    n = v.numel()
    out = torch.empty((n + _ROW - 1) // _ROW, 2, dtype=torch.int64, device=v.device)
    step = _TORCH_ROWS * _ROW
    z = torch.empty(min(step, n), dtype=torch.int64, device=v.device)
    tmp = torch.empty_like(z)
    pos = torch.arange(1, z.numel() + 1, dtype=torch.int64, device=v.device)
    r = 0
    for o in range(0, n, step):
        c = v[o:o + step]
        k = c.numel()
        zz, tt = z[:k], tmp[:k]
        torch.add(pos[:k], o, out=zz)
        zz.mul_(_GOLDEN).bitwise_xor_(c)
        for shift, mul in ((30, _MIX1), (27, _MIX2), (31, None)):
            torch.bitwise_right_shift(zz, shift, out=tt)  # arithmetic: mask the sign copies away
            zz.bitwise_xor_(tt.bitwise_and_((1 << (64 - shift)) - 1))
            if mul is not None:
                zz.mul_(mul)
        full = k // _ROW
        if full:
            torch.sum(c[:full * _ROW].view(full, _ROW), 1, out=out[r:r + full, 0])
            torch.sum(zz[:full * _ROW].view(full, _ROW), 1, out=out[r:r + full, 1])
            r += full
        if k > full * _ROW:
            out[r, 0] = c[full * _ROW:].sum()
            out[r, 1] = zz[full * _ROW:].sum()
            r += 1
    return out


def _digest_kernel(build=True):
    """The extension with `state_digest` (one HBM pass for all of a device's tensors) and
    `state_digest_cpu`, or None. build=False: only one that is loaded or importable as it is
    (CPU state never waits for a compile)."""
    try:
        from devspace_amd.ops import fused

        if build:
            e = fused.ext()
        else:
            e = fused._ext
            if e is None:
                from devspace_amd.ops import _fused_ops as e  # noqa: N813 - an in-tree build, if any

                fused._check_source(e)
        return e if e is not None and hasattr(e, "state_digest_cpu") else None
    except Exception:  # no extension in this image, or a stale build: the torch path
        return None


def digests(tensors) -> list:
    """A content digest per tensor (dtype, shape and bytes), for finding the tensors that are the
    same on several ranks (DDP replicas: parameters, optimizer moments, buffers).

    The bytes are read as int64 words in rows of 64 Ki words; each row gives two sums, a plain one
    and one of every word mixed with its position (`_digest_rows_torch`). The position term makes
    it content-exact for practical purposes: two tensors whose words are a permutation of each
    other, or differ by changes that cancel in the plain sum, get different digests (probability
    of a collision 2^-64 per row). The last bytes that do not fill a word go in raw. Device
    tensors are reduced where they live, by the gfx950 kernel in one HBM read when the fused-ops
    extension is there, and move to the host in ONE copy per device, hashed there (BLAKE2b)."""
    import torch

    words, tails = [], []
    for t in tensors:
        t = t.detach()
        if not t.is_contiguous():
            t = t.contiguous()
        b = t.reshape(-1).view(torch.uint8)
        n = b.numel()
        n8 = n // 8 * 8
        try:
            v = b[:n8].view(torch.int64)
            if v.numel() and v.data_ptr() % 8:
                raise RuntimeError("unaligned")
        except RuntimeError:  # a view at an offset that is not 8-byte aligned
            b = b.clone()
            v = b[:n8].view(torch.int64)
        words.append(v)
        tails.append(b[n8:].to(torch.int64) if n > n8 else None)
    # per device: one launch (or the torch path), one copy to the host
    rows = [None] * len(words)
    by_dev = {}
    for i, v in enumerate(words):
        by_dev.setdefault(v.device, []).append(i)
    kernel = _digest_kernel(build=any(d.type == "cuda" for d in by_dev))
    for dev, idx in by_dev.items():
        live = [i for i in idx if words[i].numel()]
        if kernel is not None and live and dev.type in ("cuda", "cpu"):
            run = kernel.state_digest if dev.type == "cuda" else kernel.state_digest_cpu
            flat = run([words[i] for i in live])
            counts = [(words[i].numel() + _ROW - 1) // _ROW for i in live]
        else:
            parts = [_digest_rows_torch(words[i]) for i in live]
            counts = [p.shape[0] for p in parts]
            flat = torch.cat(parts) if parts else None
        pieces = [flat.view(-1)] if flat is not None else []
        pieces += [tails[i] for i in idx if tails[i] is not None]
        host = torch.cat([p.to(dev) for p in pieces]).cpu().numpy() if pieces else None
        off = 0
        for i, k in zip(live, counts):
            rows[i] = host[off * 2:(off + k) * 2].tobytes()
            off += k
        off *= 2
        for i in idx:
            if tails[i] is not None:
                k = tails[i].numel()
                rows[i] = (rows[i] or b"") + host[off:off + k].tobytes()
                off += k
    out = []
    for t, r in zip(tensors, rows):
        h = hashlib.blake2b(digest_size=16)
        h.update(f"{t.dtype}|{tuple(t.shape)}|".encode())
        h.update(r or b"")
        out.append(h.hexdigest())
    return out


def plan_layout(gathered, align=64):
    """Which rank writes which tensor, and where: every rank computes the same plan from the same
    all-gathered list. `gathered[r]` is rank r's [(nbytes, digest)] in its tensor order (None:
    that rank has nothing to offer). A tensor several ranks hold (same digest) is written once,
    by the holder with the fewest bytes assigned so far, largest tensors first (round-robin by
    bytes); a tensor held twice by one rank (tied weights) is written once too.

    Returns ({digest: (owner rank, offset in its file)}, [file size per rank])."""
    holders, order = {}, []
    for r, keys in enumerate(gathered):
        for nbytes, key in keys or ():
            if key not in holders:
                holders[key] = set()
                order.append((nbytes, key))
            holders[key].add(r)
    load = [0] * len(gathered)
    where = {}
    for nbytes, key in sorted(order, key=lambda x: -x[0]):  # stable: first appearance breaks ties
        o = min(holders[key], key=lambda r: (load[r], r))
        where[key] = (o, load[o])
        load[o] += (nbytes + align - 1) // align * align
    return where, load


class Rescue:
    """Training state that survives a restart of the group.

    The reference's restart-per-change model (nodemon, redeploy) starts every process from
    nothing, which is right for a web app and ruinous for a training run: a rank failure an
    hour in would cost the hour. Every `every_s` seconds (rank 0's clock, decided at a step
    boundary for all ranks together) the ranks copy their state into shared memory
    (`rank<r>-step<N>.bin` raw tensor bytes + `.json` layout, written under temp names and
    renamed); once every rank wrote step N the older snapshots are dropped. A group started
    after a failure runs `setup()` and then loads the newest step that every rank holds, with
    the same SETUP_VERSION; a restore that fails on any rank runs `setup()` again everywhere.

    Replicated state is written once: the ranks all-gather a digest per tensor (`digests`) and
    a tensor that several ranks hold (DDP: the parameters, the optimizer moments, the buffers —
    nearly all of it) is written by one of them, spread over the ranks by bytes (`plan_layout`).
    A rank's layout points into the other ranks' files for those; restoring reads them straight
    from there (the ranks of a pod share its /dev/shm). So 8 DDP ranks with 20 GiB of state each
    need 20 GiB of shared memory, not 160, and each writes 2.5 GiB. Digests are taken at every
    snapshot (state that was equal once may diverge: a per-rank accumulator, ZeRO shards).

    HBM staging (MI355X: 288 GB per GPU): when HBM holds a copy of the tensors this rank writes,
    the snapshot is a device-to-device copy on the training stream (well under a millisecond for
    the example's 384 MiB) and a background thread streams that copy to shared memory on a side
    stream while training goes on. Training pauses only for the device copy; the ranks agree that
    every writer finished (two flags of the step-boundary all-reduce) before the older snapshots
    are dropped. "Room" is memory the next steps will not need (`hbm_budget`). When the room holds
    only part of it (a job near the HBM capacity), the largest device tensors that fit are staged
    and only the rest is copied to shared memory at the boundary, so the pause shrinks by what was
    staged. Without room (less than MIN_STAGE, or on CPU) the whole copy is made at the boundary.

    What is captured: a module's own `snapshot(ctx, state) -> obj` / `restore(ctx, state, obj)`
    when it defines them; otherwise, of a dict state, every entry with `state_dict()` /
    `load_state_dict()` (modules, DDP, optimizers, schedulers, grad scalers), plain tensors and
    scalars. Tensors come back on the device they were on (cuda → this rank's GPU)."""

    ALIGN = 64
    MIN_STAGE = 256 << 20  # HBM room below this stages nothing: the whole snapshot is copied at the boundary

    def __init__(self, root: str, rank: int, every_s: float, agree=None):
        self.root = root
        self.rank = rank
        self.every_s = every_s
        self.agree = agree  # the group's Agreement (world > 1): the digests are all-gathered over it
        self.last = time.monotonic()
        self.last_step = 0
        self.disabled = None  # why snapshots stopped for good
        self.inflight = None  # the snapshot being written (see begin / finish)
        self.staging = os.environ.get("DEVSPACE_RESCUE_STAGING", "1") != "0"
        self._side = None  # the writer's HIP stream
        self.recycle = os.environ.get("DEVSPACE_RESCUE_RECYCLE", "1") != "0"
        os.makedirs(root, exist_ok=True)

    # -- capture / apply ------------------------------------------------------------------
    @staticmethod
    def capture(mod, ctx, state):
        import torch

        if hasattr(mod, "snapshot"):
            return mod.snapshot(ctx, state)
        if not isinstance(state, dict):
            return None
        out = {}
        for k, v in state.items():
            if callable(getattr(v, "state_dict", None)) and callable(getattr(v, "load_state_dict", None)):
                out[k] = v.state_dict()
            elif isinstance(v, torch.Tensor) or v is None or isinstance(v, (bool, int, float, str)):
                out[k] = v
        return out or None

    @staticmethod
    def apply(mod, ctx, state, snap):
        import torch

        if hasattr(mod, "restore"):
            r = mod.restore(ctx, state, snap)
            return state if r is None else r
        for k, v in snap.items():
            cur = state.get(k)
            if callable(getattr(cur, "load_state_dict", None)) and isinstance(v, dict):
                cur.load_state_dict(v)
            elif isinstance(cur, torch.Tensor) and isinstance(v, torch.Tensor):
                if cur.shape != v.shape:
                    raise ValueError(f"state[{k!r}]: shape {tuple(cur.shape)} now, {tuple(v.shape)} in the snapshot")
                with torch.no_grad():
                    cur.copy_(v)
            elif k in state:
                state[k] = v
        return state

    @classmethod
    def _encode(cls, obj, tensors):
        import torch

        if isinstance(obj, torch.Tensor):
            tensors.append(obj)
            return {"T": len(tensors) - 1}
        if isinstance(obj, dict):
            return {"D": [[cls._encode(k, tensors), cls._encode(v, tensors)] for k, v in obj.items()]}
        if isinstance(obj, tuple):
            return {"U": [cls._encode(v, tensors) for v in obj]}
        if isinstance(obj, list):
            return [cls._encode(v, tensors) for v in obj]
        if obj is None or isinstance(obj, (bool, int, float, str)):
            return obj
        raise RescueSkipped(f"cannot snapshot a {type(obj).__name__} (define snapshot()/restore())")

    @classmethod
    def _decode(cls, obj, tensors):
        if isinstance(obj, list):
            return [cls._decode(v, tensors) for v in obj]
        if isinstance(obj, dict):
            if "T" in obj:
                return tensors[obj["T"]]
            if "U" in obj:
                return tuple(cls._decode(v, tensors) for v in obj["U"])
            return {cls._decode(k, tensors): cls._decode(v, tensors) for k, v in obj["D"]}
        return obj

    # -- files -----------------------------------------------------------------------------
    def _path(self, step, ext, rank=None):
        return os.path.join(self.root, f"rank{self.rank if rank is None else rank}-step{step}.{ext}")

    def _spare(self) -> str:
        return os.path.join(self.root, f"rank{self.rank}-spare.bin")

    def _spare_bytes(self) -> int:
        """Shared memory the group's spare files hold (each is reused by its rank's next write)."""
        n = 0
        for name in os.listdir(self.root):
            if re.match(r"rank\d+-spare\.bin$", name):
                try:
                    n += os.path.getsize(os.path.join(self.root, name))
                except OSError:
                    pass
        return n

    def due(self, step: int) -> bool:
        return (self.every_s > 0 and self.disabled is None and self.inflight is None and step > self.last_step
                and time.monotonic() - self.last >= self.every_s)

    @staticmethod
    def hbm_room(nbytes, free, reserved, peak, margin=256 << 20) -> bool:
        """Room in HBM for a staged copy of `nbytes` that the next steps do not need.

        free: what the driver has not handed out; reserved: what PyTorch's caching allocator
        holds (in use or cached); peak: the most the steps allocated at once since the last
        snapshot finished (max_memory_allocated, reset then). The steps will again need `peak`
        out of `reserved + free` while the copy is alive (the background writer may take several
        steps): what is left is free + reserved - peak. (Counting all cached memory as room, as
        round 4 did, handed the copy the activation memory of the next step: a run within one
        state size of the HBM capacity went out of memory in step().)"""
        return free + reserved - peak >= nbytes * 1.1 + margin

    @staticmethod
    def hbm_budget(free, reserved, peak, margin=256 << 20) -> int:
        """The largest staged copy hbm_room allows: bytes of HBM the next steps do not need."""
        return max(0, int((free + reserved - peak - margin) / 1.1))

    def _hbm_budget(self, device) -> int:
        import torch

        try:
            free, _ = torch.cuda.mem_get_info(device)
            reserved = torch.cuda.memory_reserved(device)
            peak = torch.cuda.max_memory_allocated(device)
        except RuntimeError:  # no answer from the runtime: copy at the boundary instead
            return 0
        return self.hbm_budget(free, reserved, peak)

    def steady(self, device) -> None:
        """Training is past its start-up: the step's peak is measured from here (the staging
        decision must not count setup()'s transient allocations, nor a staged copy of ours)."""
        if device is not None and device.type == "cuda":
            import torch

            try:
                torch.cuda.reset_peak_memory_stats(device)
            except RuntimeError:
                pass

    def _plan(self, ctx, tensors):
        """This rank's part of the snapshot: (tensor metas with their file and offset, the
        indices of the tensors this rank writes with their offsets, file sizes per rank). Every
        rank of the group calls it at the same boundary (one all-gather), failing or not."""
        keys, err = None, None
        t0 = time.perf_counter()
        try:
            keys = [(t.numel() * t.element_size(), d) for t, d in zip(tensors, digests(tensors))]
            self.digest_ms = (time.perf_counter() - t0) * 1000.0
        except Exception as e:  # a device error: this rank offers nothing; the snapshot fails
            err = f"{type(e).__name__}: {e}"
        gathered = self.agree.gather(keys) if self.agree is not None else [keys]
        if err is not None:
            raise RuntimeError(f"digest: {err}")
        bad = [r for r, k in enumerate(gathered) if k is None]
        if bad:
            raise RescueSkipped(f"rank {bad[0]} could not digest its state")
        where, load = plan_layout(gathered, self.ALIGN)
        metas, mine, seen = [], [], set()
        for i, (t, (nbytes, key)) in enumerate(zip(tensors, keys)):
            owner, off = where[key]
            metas.append({"dtype": str(t.dtype).replace("torch.", ""), "shape": list(t.shape),
                          "device": t.device.type, "file": owner, "offset": off, "nbytes": nbytes})
            if owner == self.rank and key not in seen:
                seen.add(key)
                mine.append((i, off, nbytes))
        return metas, mine, load

    def begin(self, mod, ctx, state, gen, setup_version) -> None:
        """Starts this rank's part of the snapshot of `state` at ctx.step (self.inflight): staged
        in HBM and written by a background thread, or written here. Errors end up in the job,
        never raised: every rank must reach the next boundary with a job to agree on (and, with
        several ranks, make the digest all-gather)."""
        import shutil

        import torch

        t0 = time.perf_counter()
        job = {"step": ctx.step, "gen": gen, "bytes": 0, "total": 0, "state_bytes": 0, "err": None, "done": False,
               "staged": False, "pause_ms": 0.0, "write_ms": 0.0}
        self.inflight = job
        tensors, tree, enc_err = [], None, None
        try:
            tree = self._encode(self.capture(mod, ctx, state), tensors)
        except Exception as e:  # RescueSkipped (an unsupported type), an error in the user's hook
            enc_err = e
            tensors = []
        try:
            metas, mine, load = self._plan(ctx, tensors)  # (collective: before any early exit)
            if enc_err is not None:
                raise enc_err
            job["bytes"], job["total"] = load[self.rank], sum(load)
            job["state_bytes"] = sum(m["nbytes"] for m in metas)
            # the ranks of the pod write theirs into the same /dev/shm at the same time
            free = shutil.disk_usage(self.root).free + self._spare_bytes()
            if job["total"] > free * 0.9:
                raise RescueSkipped(f"{self.root} has {free >> 20} MiB free, the group's snapshot needs "
                                    f"{job['total'] >> 20} MiB")
            files = {str(r): load[r] for r in sorted({m["file"] for m in metas} | {self.rank})}
            meta = {"step": ctx.step, "gen": gen, "setup_version": setup_version, "world": ctx.world_size,
                    "time": time.time(), "bytes": load[self.rank], "files": files, "tensors": metas, "tree": tree}
            own = [(tensors[i], off, n) for i, off, n in mine]
            dev_bytes = sum(n for t, _, n in own if t.device.type == "cuda")
            budget = 0
            if self.staging and dev_bytes and ctx.device.type == "cuda":
                budget = self._hbm_budget(ctx.device)
            if budget >= dev_bytes:  # (also: nothing on the device) everything is staged
                staged, rest = list(own) if budget else [], [] if budget else list(own)
            else:
                # HBM holds part of it: stage the largest device tensors that fit, copy the rest
                # at the boundary (the pause shrinks by what is staged)
                staged, rest, left = [], [], budget
                for t, off, n in sorted(own, key=lambda x: -x[2]):
                    if t.device.type == "cuda" and n <= left and budget >= self.MIN_STAGE:
                        staged.append((t, off, n))
                        left -= n
                    else:
                        rest.append((t, off, n))
            if staged:
                # the file is sized and mapped at the boundary only for a part written there; else
                # the background writer does it (a fresh 2 GiB file is 119-272 ms of fallocate)
                part = self._open(ctx.step, meta["bytes"]) if rest else None
                try:
                    if rest:  # the live tensors the background write cannot see unchanged
                        self._fill(part, [(t.detach(), off, n) for t, off, n in rest])
                        job["boundary_bytes"] = sum(n for _, _, n in rest)
                    boundary_ms = (time.perf_counter() - t0) * 1000.0
                    start, end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    with torch.no_grad():
                        start.record()
                        copies = [(t.detach().clone(), off, n) for t, off, n in staged]  # host tensors change too
                        end.record()
                except BaseException:
                    if part is not None:
                        self._close(part)
                    raise
                job["staged"] = True
                job["staged_bytes"] = sum(n for _, _, n in staged)
                job["thread"] = threading.Thread(target=self._write_job, name="devspace-rescue-writer", daemon=True,
                                                 args=(job, copies, meta, ctx.device, (start, end), part,
                                                       boundary_ms if rest else 0.0))
                job["thread"].start()
            else:
                self._write_job(job, [(t.detach(), off, n) for t, off, n in own], meta, None, None)
                job["pause_ms"] = (time.perf_counter() - t0) * 1000.0
        except Exception as e:  # RescueSkipped, an unsupported type in the state, a device error
            job["err"] = str(e) if isinstance(e, RescueSkipped) else f"{type(e).__name__}: {e}"
            job["done"] = True

    def _write_job(self, job, own, meta, device, events, part=None, boundary_ms=0.0) -> None:
        import torch

        t0 = time.perf_counter()
        try:
            if events is not None:
                torch.cuda.set_device(device)  # this thread's current device (HIP's is per thread)
                if self._side is None:
                    self._side = torch.cuda.Stream(device=device)
                self._side.wait_event(events[1])
                with torch.cuda.stream(self._side):
                    self._write(job["step"], own, meta, part)
                job["pause_ms"] = boundary_ms + events[0].elapsed_time(events[1])
            else:
                self._write(job["step"], own, meta, part)
        except Exception as e:  # shared memory full (SIGBUS is not an exception: sized above), I/O
            job["err"] = f"{type(e).__name__}: {e}"
        finally:
            del own[:]  # the HBM copies go back to the caching allocator
            job["write_ms"] = (time.perf_counter() - t0) * 1000.0
            job["done"] = True

    def _open(self, step, size):
        """This rank's data file of `step` (as .tmp), sized and mapped: [file, mapping or None,
        uint8 tensor over it or None, step]."""
        import torch

        binp = self._path(step, "bin")
        fresh = True
        try:  # the superseded snapshot's file: its shared-memory pages are allocated already
            os.replace(self._spare(), binp + ".tmp")
            fresh = False
        except OSError:
            pass
        f = open(binp + ".tmp", "w+b" if fresh else "r+b")
        try:
            have = 0 if fresh else os.fstat(f.fileno()).st_size
            if have > size:
                os.ftruncate(f.fileno(), size)
            elif have < size:
                # reserve the pages first: a full tmpfs then fails here (ENOSPC), not as a SIGBUS
                # on a store into the mapping
                os.posix_fallocate(f.fileno(), have, size - have)
            if not size:
                return [f, None, None, step]
            # MAP_POPULATE: the pages are mapped in one call, not one fault per 4 KiB store
            mm = mmap.mmap(f.fileno(), size, flags=mmap.MAP_SHARED | getattr(mmap, "MAP_POPULATE", 0))
        except BaseException:
            f.close()
            raise
        return [f, mm, torch.frombuffer(mm, dtype=torch.uint8), step]

    @staticmethod
    def _fill(part, own) -> None:
        """One copy per tensor, device (or host) straight into the mapped shared memory. (Through
        a pinned bounce pair, as restores go, the runner's writes were slower: 934-1077 ms against
        436-588 ms for 2.5 GB at the boundary on the MI355X box.)"""
        buf = part[2]
        for t, off, n in own:
            if n:
                buf[off:off + n].view(t.dtype).view(t.shape).copy_(t)

    @staticmethod
    def _close(part) -> None:
        f, mm = part[0], part[1]
        part[2] = None
        if mm is not None:
            _close_mapping(mm)
        f.close()

    def _write(self, step, own, meta, part=None) -> None:
        import json

        part = part if part is not None else self._open(step, meta["bytes"])
        try:
            if own:
                self._fill(part, own)
        finally:
            self._close(part)
        binp, jsp = self._path(step, "bin"), self._path(step, "json")
        with open(jsp + ".tmp", "w") as f:
            json.dump(meta, f)
        os.replace(binp + ".tmp", binp)
        os.replace(jsp + ".tmp", jsp)  # the layout last: its presence marks a complete part

    def commit(self, step: int, ok: bool) -> None:
        """Every rank wrote `step` (ok): drop this rank's older files; else drop this one. The
        newest superseded data file is kept as the spare the next snapshot is written into (its
        pages are allocated: a fresh 2 GiB file cost 119-272 ms of posix_fallocate on the
        MI355X box), while the shared memory has room for another snapshot of its size besides."""
        import shutil

        for name in sorted(os.listdir(self.root), key=lambda x: -int((re.search(r"-step(\d+)\.", x) or [0, 0])[1])):
            m = re.match(rf"rank{self.rank}-step(\d+)\.(bin|json)(\.tmp)?$", name)
            if m and (int(m.group(1)) != step if ok else int(m.group(1)) == step):
                path = os.path.join(self.root, name)
                try:
                    if (ok and m.group(2) == "bin" and not m.group(3) and self.recycle
                            and not os.path.exists(self._spare())
                            and shutil.disk_usage(self.root).free >= os.path.getsize(path)):
                        os.replace(path, self._spare())
                    else:
                        os.unlink(path)
                except OSError:
                    pass
        if ok:
            self.last_step = step
        self.last = time.monotonic()

    def _files_of(self, meta, step) -> dict:
        """{rank: (path, size)} of the files a layout reads (round-4 layouts: the rank's own)."""
        files = meta.get("files") or {str(self.rank): meta["bytes"]}
        return {int(r): (self._path(step, "bin", int(r)), n) for r, n in files.items()}

    def available(self, setup_version, world) -> list:
        """Steps whose layout this rank holds, for this SETUP_VERSION and world size, with every
        file the layout points into complete."""
        import json

        steps = []
        for name in os.listdir(self.root):
            m = re.match(rf"rank{self.rank}-step(\d+)\.json$", name)
            if not m:
                continue
            step = int(m.group(1))
            try:
                with open(os.path.join(self.root, name)) as f:
                    meta = json.load(f)
                ok = all(os.path.getsize(p) == n for p, n in self._files_of(meta, step).values())
            except (OSError, ValueError, KeyError):
                continue
            if ok and meta.get("setup_version") == setup_version and meta.get("world") == world:
                steps.append(step)
        return sorted(steps)

    def load(self, step, device):
        """(state tree with tensors materialised, metadata) of this rank's snapshot `step`; the
        tensors another rank wrote come straight from its file."""
        import json

        import torch

        with open(self._path(step, "json")) as f:
            meta = json.load(f)
        maps, bufs, tensors = {}, {}, []
        try:
            for r, (path, size) in self._files_of(meta, step).items():
                with open(path, "rb") as f:
                    if os.fstat(f.fileno()).st_size != size:
                        raise ValueError(f"snapshot step={step} of rank {r} is truncated")
                    if size:
                        maps[r] = mmap.mmap(f.fileno(), size, access=mmap.ACCESS_COPY)
                        bufs[r] = torch.frombuffer(maps[r], dtype=torch.uint8)
            for m in meta["tensors"]:
                dtype = getattr(torch, m["dtype"])
                if not m["nbytes"]:
                    tensors.append(torch.empty(m["shape"], dtype=dtype))
                    continue
                r = m.get("file", self.rank)
                src = bufs[r][m["offset"]:m["offset"] + m["nbytes"]].view(dtype).view(m["shape"])
                # own memory either way (the mappings are closed below)
                on_gpu = m["device"] == "cuda" and device.type == "cuda"
                if on_gpu and m["nbytes"] >= _BOUNCE_MIN:
                    out = torch.empty(m["shape"], dtype=dtype, device=device)
                    _h2d(out, bufs[r][m["offset"]:m["offset"] + m["nbytes"]])
                    tensors.append(out)
                else:
                    tensors.append(src.to(device) if on_gpu else src.clone())
                del src
        finally:
            bufs.clear()
            for mm in maps.values():
                _close_mapping(mm)
        return self._decode(meta["tree"], tensors), meta


def _rescue_finish(rescue, ctx, failed: bool) -> None:
    """Every rank's writer is done (agreed at a boundary): keep this snapshot and drop the older
    ones, or — it failed on some rank — drop it and stop taking snapshots, on every rank alike."""
    job, rescue.inflight = rescue.inflight, None
    rescue.commit(job["step"], not failed)
    if job["staged"]:  # the staged copy is gone: the next decision measures the steps alone
        rescue.steady(ctx.device)
    if failed:
        why = job["err"] or "failed on another rank"
        rescue.disabled = why
        if job["err"]:
            ctx.error(f"rescue snapshot step={job['step']} failed: {job['err']}")
        ctx.log(f"rescue snapshots off ({why})")
        return
    how = "staged in HBM, written in the background" if job["staged"] else "written at the step boundary"
    if job["staged"] and job.get("boundary_bytes"):
        how = (f"{job['staged_bytes'] / 2**20:.0f} MiB staged in HBM, {job['boundary_bytes'] / 2**20:.0f} MiB "
               f"copied at the step boundary, written in the background")
    ctx.log(f"rescue snapshot step={job['step']} gen={job['gen']} {job['bytes'] / 2**20:.1f} MiB/rank: "
            f"training paused {job['pause_ms']:.2f} ms, {how} in {job['write_ms']:.1f} ms "
            f"(group: {job['total'] / 2**20:.1f} MiB in shared memory for "
            f"{job['state_bytes'] * ctx.world_size / 2**20:.1f} MiB of state on {ctx.world_size} rank(s); "
            f"digest {getattr(rescue, 'digest_ms', 0.0):.1f} ms)")


def _rescue_final(rescue, agree, mod, ctx, state, gen, setup_version) -> None:
    """Stopping with an explicit --rescue-dir (a volume that outlives the pod): the snapshot in
    flight is finished and one more is taken where training stopped, so the next start — a new
    pod after `devspace purge`, tomorrow — resumes at that step."""
    def settle():
        job = rescue.inflight
        if job is None:
            return
        if job.get("thread") is not None:
            job["thread"].join()
        errs = agree.gather(job["err"]) if agree is not None else [job["err"]]
        _rescue_finish(rescue, ctx, any(e is not None for e in errs))

    settle()
    if rescue.disabled is None and ctx.step > rescue.last_step:  # the same decision on every rank
        ctx.log(f"stopping: a last rescue snapshot at step={ctx.step} in {rescue.root}")
        rescue.begin(mod, ctx, state, gen, setup_version)
        settle()


def _rescue_restore(rescue, agree, mod, ctx, state):
    """After setup() of a (re)started group: the newest snapshot every rank holds for this
    SETUP_VERSION, loaded on every rank, or none at all."""
    setup_version = getattr(mod, "SETUP_VERSION", None)
    steps = rescue.available(setup_version, ctx.world_size)
    held = agree.gather(steps) if agree is not None else [steps]
    common = set(held[0]).intersection(*[set(h) for h in held[1:]])
    if not common:
        if any(held):
            ctx.log("rescue: no snapshot that every rank holds for this SETUP_VERSION: starting from setup()")
        return state
    step = max(common)
    t0 = time.perf_counter()
    err, meta = None, None
    try:
        snap, meta = rescue.load(step, ctx.device)
        state = rescue.apply(mod, ctx, state, snap)
    except Exception as e:
        err = f"{type(e).__name__}: {e}"
    errs = agree.gather(err) if agree is not None else [err]
    bad = [(r, e) for r, e in enumerate(errs) if e is not None]
    if bad:
        # some ranks may hold half-restored state: every rank starts over from setup()
        ctx.log(f"rescue: snapshot step={step} did not restore on rank {bad[0][0]} ({bad[0][1]}): "
                f"starting from setup()")
        return mod.setup(ctx)
    ctx.step = step
    rescue.last_step, rescue.last = step, time.monotonic()
    nbytes = sum(m["nbytes"] for m in meta["tensors"])
    ctx.log(f"restored step={step} gen={meta['gen']} from the rescue snapshot (age {time.time() - meta['time']:.1f} s, "
            f"{nbytes / 2**20:.1f} MiB/rank in {(time.perf_counter() - t0) * 1000.0:.1f} ms)")
    return state


def _in_pod() -> bool:
    return bool(os.environ.get("KUBERNETES_SERVICE_HOST"))


def _default_rescue_dir(entry: str, nproc: int) -> str:
    """In a pod: one directory per entry file and rank count in /dev/shm, the pod's memory
    volume, so a container that the kubelet restarts (an OOM kill, a crash of the runner itself)
    finds the snapshots its previous run left. Elsewhere: this process's own (a later run on the
    same machine starts fresh)."""
    import tempfile

    base = os.environ.get("DEVSPACE_RESCUE_ROOT") or (
        "/dev/shm" if os.path.isdir("/dev/shm") and os.access("/dev/shm", os.W_OK) else tempfile.gettempdir())
    if _in_pod():
        key = hashlib.sha256(f"{os.path.abspath(entry)}|{nproc}".encode()).hexdigest()[:12]
        return os.path.join(base, f"devspace-rescue-{key}")
    # what runners killed outright (SIGKILL: no clean-up) left behind here
    for name in os.listdir(base):
        m = re.match(r"devspace-rescue-(\d+)$", name)
        if m and not os.path.exists(f"/proc/{m.group(1)}"):
            _drop_rescue_dir(os.path.join(base, name))
    return os.path.join(base, f"devspace-rescue-{os.getpid()}")


def _drop_rescue_dir(path: str) -> None:
    import shutil

    shutil.rmtree(path, ignore_errors=True)
