"""The runner's rescue snapshots (devspace_amd/runner.py `Rescue`) round-trip what a training
state holds: module and optimizer state dicts (int keys, tuples, 0-dim step tensors), plain
tensors of any dtype and layout (bf16, bool, empty, non-contiguous), Python numbers and strings;
a module's own snapshot()/restore() hooks win; a state it cannot serialise turns snapshots off
with a reason instead of failing the step."""

import os
import types

import pytest
import torch

from devspace_amd import runner


def _ctx(step=7, world=1):
    ctx = runner.Context(0, world, 0, torch.device("cpu"))
    ctx.step = step
    return ctx


def _state(seed):
    torch.manual_seed(seed)
    model = torch.nn.Sequential(torch.nn.Linear(8, 8), torch.nn.LayerNorm(8)).to(torch.bfloat16)
    opt = torch.optim.AdamW(model.parameters(), lr=1e-3, betas=(0.8, 0.95))
    model(torch.randn(4, 8, dtype=torch.bfloat16)).float().pow(2).mean().backward()
    opt.step()
    return {"model": model, "opt": opt,
            "t": torch.randn(6, 4).t(),  # non-contiguous
            "mask": torch.rand(5) > 0.5, "empty": torch.zeros(0, 3), "scalar": torch.tensor(3.5),
            "n": 41, "lr_scale": 0.5, "name": "run-a", "none": None,
            "loader": object()}  # not snapshotable without hooks: left out, not an error


def _take(rescue, mod, ctx, state):
    rescue.begin(mod, ctx, state, gen=3, setup_version=1)
    job = rescue.inflight
    if job.get("thread") is not None:
        job["thread"].join()
    runner._rescue_finish(rescue, ctx, job["err"] is not None)
    return job


def test_round_trip_of_a_training_state(tmp_path):
    mod = types.SimpleNamespace()
    r = runner.Rescue(str(tmp_path), 0, every_s=60)
    src = _state(0)
    job = _take(r, mod, _ctx(), src)
    assert job["err"] is None and job["bytes"] > 0 and not job["staged"]  # CPU: written at the boundary
    assert r.available(1, 1) == [7] and r.available(2, 1) == [] and r.available(1, 2) == []
    dst = _state(1)
    snap, meta = r.load(7, torch.device("cpu"))
    dst = runner.Rescue.apply(mod, _ctx(), dst, snap)
    for a, b in zip(src["model"].state_dict().values(), dst["model"].state_dict().values()):
        assert a.dtype == b.dtype == torch.bfloat16 and torch.equal(a, b)
    so, do = src["opt"].state_dict(), dst["opt"].state_dict()
    assert do["param_groups"][0]["betas"] == (0.8, 0.95)  # tuples stay tuples
    assert set(do["state"]) == set(so["state"]) and all(isinstance(k, int) for k in do["state"])
    for k in so["state"]:
        for name, v in so["state"][k].items():
            assert torch.equal(v, do["state"][k][name]), (k, name)
    assert torch.equal(dst["t"], src["t"]) and torch.equal(dst["mask"], src["mask"])
    assert dst["empty"].shape == (0, 3) and float(dst["scalar"]) == 3.5
    assert (dst["n"], dst["lr_scale"], dst["name"], dst["none"]) == (41, 0.5, "run-a", None)
    assert meta["gen"] == 3 and meta["step"] == 7


def test_newer_snapshot_replaces_the_older_one(tmp_path):
    mod = types.SimpleNamespace()
    r = runner.Rescue(str(tmp_path), 0, every_s=60)
    _take(r, mod, _ctx(step=7), _state(0))
    _take(r, mod, _ctx(step=9), _state(0))
    assert r.available(1, 1) == [9]
    # the superseded data file stays as the spare the next snapshot is written into
    assert sorted(p.name for p in tmp_path.iterdir()) == ["rank0-spare.bin", "rank0-step9.bin", "rank0-step9.json"]
    _take(r, mod, _ctx(step=11), _state(0))
    assert r.available(1, 1) == [11]
    assert sorted(p.name for p in tmp_path.iterdir()) == ["rank0-spare.bin", "rank0-step11.bin", "rank0-step11.json"]
    snap, _ = r.load(11, torch.device("cpu"))  # written into the recycled file: intact
    assert torch.equal(snap["t"], _state(0)["t"])


def test_no_spare_is_kept_without_room_for_another_snapshot(tmp_path, monkeypatch):
    """The superseded file is kept for the next write only while /dev/shm could hold another
    snapshot of its size besides (others — DataLoader workers, RCCL — share it); and never with
    DEVSPACE_RESCUE_RECYCLE=0."""
    import collections
    import shutil

    mod = types.SimpleNamespace()
    r = runner.Rescue(str(tmp_path / "full"), 0, every_s=60)
    real = shutil.disk_usage
    _take(r, mod, _ctx(step=7), _state(0))
    usage = collections.namedtuple("u", "total used free")
    frees = iter([1 << 30, 100])  # begin's room check: room; commit's check for a spare: none
    monkeypatch.setattr(shutil, "disk_usage", lambda p: usage(1 << 31, 1 << 30, next(frees)))
    _take(r, mod, _ctx(step=9), _state(0))
    monkeypatch.setattr(shutil, "disk_usage", real)
    assert sorted(p.name for p in (tmp_path / "full").iterdir()) == ["rank0-step9.bin", "rank0-step9.json"]
    monkeypatch.setenv("DEVSPACE_RESCUE_RECYCLE", "0")
    r2 = runner.Rescue(str(tmp_path / "off"), 0, every_s=60)
    _take(r2, mod, _ctx(step=7), _state(0))
    _take(r2, mod, _ctx(step=9), _state(0))
    assert sorted(p.name for p in (tmp_path / "off").iterdir()) == ["rank0-step9.bin", "rank0-step9.json"]


def test_module_hooks_win_and_unserialisable_state_turns_snapshots_off(tmp_path):
    seen = {}
    mod = types.SimpleNamespace(snapshot=lambda ctx, state: {"w": state["w"] * 2},
                                restore=lambda ctx, state, obj: seen.update(obj) or {"w": obj["w"]})
    r = runner.Rescue(str(tmp_path / "a"), 0, every_s=60)
    _take(r, mod, _ctx(), {"w": torch.ones(3)})
    snap, _ = r.load(7, torch.device("cpu"))
    out = runner.Rescue.apply(mod, _ctx(), {"w": torch.zeros(3)}, snap)
    assert torch.equal(out["w"], torch.full((3,), 2.0)) and "w" in seen
    bad = types.SimpleNamespace(snapshot=lambda ctx, state: {"f": lambda: 1})
    r2 = runner.Rescue(str(tmp_path / "b"), 0, every_s=60)
    job = _take(r2, bad, _ctx(), {})
    assert job["err"] and "cannot snapshot a function" in job["err"] and r2.disabled, job
    assert r2.available(None, 1) == []


def test_restore_into_a_changed_model_fails_cleanly(tmp_path):
    mod = types.SimpleNamespace()
    r = runner.Rescue(str(tmp_path), 0, every_s=60)
    _take(r, mod, _ctx(), {"w": torch.ones(4)})
    snap, _ = r.load(7, torch.device("cpu"))
    with pytest.raises(ValueError, match="shape"):
        runner.Rescue.apply(mod, _ctx(), {"w": torch.ones(5)}, snap)


@pytest.mark.gpu
def test_hbm_staged_snapshot_round_trip_on_the_gpu(tmp_path):
    """On the MI355X the device tensors are copied within HBM at the boundary (training pauses for
    that alone) and written by the background thread on a side stream; the step that runs
    meanwhile changes the live tensors, not the snapshot."""
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    dev = torch.device("cuda", 0)
    ctx = runner.Context(0, 1, 0, dev)
    ctx.step = 5
    torch.manual_seed(0)
    model = torch.nn.Linear(512, 512).to(dev, torch.bfloat16)
    opt = torch.optim.AdamW(model.parameters(), lr=1e-3)
    model(torch.randn(8, 512, device=dev, dtype=torch.bfloat16)).float().sum().backward()
    opt.step()
    state = {"model": model, "opt": opt, "n": 5}
    want = {k: v.detach().clone() for k, v in model.state_dict().items()}
    r = runner.Rescue(str(tmp_path), 0, every_s=60)
    r.begin(types.SimpleNamespace(), ctx, state, gen=1, setup_version=None)
    job = r.inflight
    assert job["staged"], job  # free HBM: a device copy, written in the background
    with torch.no_grad():  # the next step changes the live weights while the write goes on
        for p in model.parameters():
            p.add_(1.0)
    job["thread"].join()
    assert job["err"] is None and job["pause_ms"] < 50, job
    runner._rescue_finish(r, ctx, False)
    snap, _ = r.load(5, dev)
    fresh = {"model": torch.nn.Linear(512, 512).to(dev, torch.bfloat16),
             "opt": None, "n": 0}
    fresh["opt"] = torch.optim.AdamW(fresh["model"].parameters(), lr=1e-3)
    runner.Rescue.apply(types.SimpleNamespace(), ctx, fresh, snap)
    for k, v in fresh["model"].state_dict().items():
        assert v.is_cuda and torch.equal(v, want[k]), k  # the snapshot's values, not the later ones
    assert fresh["n"] == 5


@pytest.mark.gpu
@pytest.mark.parametrize("staging", ["0", "1"])
def test_large_device_tensors_round_trip_through_the_pinned_bounce(tmp_path, monkeypatch, staging):
    """Large device tensors, written at the boundary or from the HBM-staged copy, into a fresh file
    and then into the recycled spare, come back through two pinned 64 MiB buffers (sizes that end
    inside a chunk included); smaller and non-contiguous ones take the direct copy. Every
    snapshot restores bit-exact."""
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    from devspace_amd import rescue as rmod

    monkeypatch.setenv("DEVSPACE_RESCUE_STAGING", staging)
    dev = torch.device("cuda", 0)
    ctx = runner.Context(0, 1, 0, dev)
    torch.manual_seed(1)
    state = {"a": torch.randn(37, 1 << 20, device=dev, dtype=torch.bfloat16),  # 74 MiB: 64 + 10
             "b": torch.randn(50, 1 << 20, device=dev),  # 200 MiB: 3 x 64 + 8
             "c": torch.randn(9, 1 << 18, device=dev),  # 9 MiB: one partial chunk
             "d": torch.randn(1024, 1024, device=dev).t(),  # 4 MiB, non-contiguous: direct
             "e": torch.randint(0, 2, (3, 1 << 23), device=dev).bool()}  # 24 MiB of bool
    assert state["a"].numel() * 2 >= rmod._BOUNCE_MIN and not state["d"].is_contiguous()
    r = runner.Rescue(str(tmp_path), 0, every_s=60)
    for step in (5, 6, 7):
        ctx.step = step
        with torch.no_grad():
            for k in ("a", "b", "c", "d"):
                state[k].add_(1.0)
        want = {k: v.clone() for k, v in state.items()}
        job = _take(r, types.SimpleNamespace(), ctx, state)
        assert job["err"] is None and job["staged"] == (staging == "1"), job
        assert r.available(1, 1) == [step]
        snap, _ = r.load(step, dev)
        for k, v in want.items():
            got = snap[k]
            assert got.is_cuda and got.dtype == v.dtype and got.shape == v.shape, k
            assert torch.equal(got, v), (step, k)
    assert (tmp_path / "rank0-spare.bin").exists()  # steps 6 and 7 were written into the spare


@pytest.mark.gpu
def test_partial_hbm_staging_copies_only_the_overflow_at_the_boundary(tmp_path):
    """A job near the HBM capacity: the room holds part of the state. The largest device tensors
    that fit are staged, the rest is copied at the boundary; the step that runs while the writer
    works changes neither part of the snapshot."""
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    dev = torch.device("cuda", 0)
    ctx = runner.Context(0, 1, 0, dev)
    ctx.step = 3
    mib = 1 << 20
    state = {"a": torch.randn(75, mib, device=dev),  # 300 MiB: staged
             "b": torch.randn(50, mib, device=dev),  # 200 MiB: at the boundary
             "c": torch.randn(25, mib, device=dev),  # 100 MiB: at the boundary (does not fit after a)
             "h": torch.randn(1000)}  # host: at the boundary
    want = {k: v.clone() for k, v in state.items()}
    r = runner.Rescue(str(tmp_path), 0, every_s=60)
    r._hbm_budget = lambda device: 320 * mib
    r.begin(types.SimpleNamespace(), ctx, state, gen=1, setup_version=1)
    job = r.inflight
    assert job["staged"] and job["staged_bytes"] == 300 * mib, job
    assert job["boundary_bytes"] == 300 * mib + 4000, job
    with torch.no_grad():  # the next step
        for v in state.values():
            v.add_(1.0)
    job["thread"].join()
    assert job["err"] is None, job
    runner._rescue_finish(r, ctx, False)
    snap, _ = r.load(3, dev)
    for k, v in want.items():
        assert torch.equal(snap[k].cpu(), v.cpu()), k
    # too little room for anything worth staging: all of it at the boundary
    r2 = runner.Rescue(str(tmp_path / "b"), 0, every_s=60)
    r2._hbm_budget = lambda device: runner.Rescue.MIN_STAGE - 1
    job2 = _take(r2, types.SimpleNamespace(), ctx, state)
    assert job2["err"] is None and not job2["staged"], job2


class _ThreadGroup:
    """The Agreement's all-gather for ranks simulated as threads of one process."""

    def __init__(self, world):
        import threading

        self.world = world
        self.box = [None] * world
        self.barrier = threading.Barrier(world)

    def for_rank(self, rank):
        group = self

        class _Agree:
            def gather(self, obj):
                group.box[rank] = obj
                group.barrier.wait()
                out = list(group.box)
                group.barrier.wait()
                return out

        return _Agree()


def _ddp_like_state(rank, seed=0):
    """What DDP ranks hold: the same model and optimizer on every rank, plus a little per-rank
    state (a data-loader position, a per-rank RNG draw)."""
    torch.manual_seed(seed)
    model = torch.nn.Sequential(torch.nn.Linear(256, 256), torch.nn.Linear(256, 64))
    opt = torch.optim.AdamW(model.parameters(), lr=1e-3)
    model(torch.ones(4, 256)).sum().backward()
    opt.step()
    return {"model": model, "opt": opt, "cursor": torch.full((1000,), float(rank)), "rank": rank}


def _group_take(root, world, states, step=7):
    import threading

    g = _ThreadGroup(world)
    rescues = [runner.Rescue(str(root), r, every_s=60, agree=g.for_rank(r)) for r in range(world)]
    jobs = [None] * world

    def one(r):
        ctx = runner.Context(r, world, r, torch.device("cpu"))
        ctx.step = step
        rescues[r].begin(types.SimpleNamespace(), ctx, states[r], gen=1, setup_version=1)
        jobs[r] = rescues[r].inflight

    ts = [threading.Thread(target=one, args=(r,)) for r in range(world)]
    [t.start() for t in ts]
    [t.join() for t in ts]
    for r in range(world):
        assert jobs[r]["err"] is None, jobs[r]
        runner._rescue_finish(rescues[r], runner.Context(r, world, r, torch.device("cpu")), False)
    return rescues, jobs


def test_replicated_state_is_written_once_across_ranks(tmp_path):
    """4 ranks holding the same model and optimizer (DDP) write that state once between them,
    spread over the ranks by bytes, and each rank's own tensors once; every rank restores its
    exact state, reading the replicated tensors from the other ranks' files."""
    world = 4
    states = [_ddp_like_state(r) for r in range(world)]
    rescues, jobs = _group_take(tmp_path, world, states)
    one_rank = sum(p.numel() * p.element_size() for p in states[0]["model"].parameters()) * 3  # + 2 moments
    total = sum(os.path.getsize(tmp_path / f"rank{r}-step7.bin") for r in range(world))
    assert total == jobs[0]["total"]
    # one copy of the replicated state plus 4 cursors (and alignment), not 4 copies
    assert one_rank <= total < one_rank * 1.1 + world * 4096, (total, one_rank)
    sizes = [jobs[r]["bytes"] for r in range(world)]
    assert max(sizes) < one_rank * 0.6, sizes  # spread over the ranks, not all on rank 0
    for r in range(world):
        assert rescues[r].available(1, world) == [7]
        snap, _ = rescues[r].load(7, torch.device("cpu"))
        fresh = _ddp_like_state(r, seed=99)
        fresh["rank"] = -1
        fresh = runner.Rescue.apply(types.SimpleNamespace(), None, fresh, snap)
        for a, b in zip(states[r]["model"].state_dict().values(), fresh["model"].state_dict().values()):
            assert torch.equal(a, b)
        so, fo = states[r]["opt"].state_dict()["state"], fresh["opt"].state_dict()["state"]
        for k in so:
            for name in so[k]:
                assert torch.equal(so[k][name], fo[k][name]), (k, name)
        assert torch.equal(fresh["cursor"], states[r]["cursor"]) and fresh["rank"] == r


def test_a_rank_whose_state_diverged_writes_its_own(tmp_path):
    """Digests are taken at every snapshot: a tensor that differs on one rank (a per-rank
    accumulator, a shard) is written by that rank, not taken from a replica."""
    world = 2
    states = [_ddp_like_state(r) for r in range(world)]
    with torch.no_grad():
        next(iter(states[1]["model"].parameters()))[0, 0] += 1.0
    rescues, _ = _group_take(tmp_path, world, states)
    for r in range(world):
        snap, _ = rescues[r].load(7, torch.device("cpu"))
        fresh = runner.Rescue.apply(types.SimpleNamespace(), None, _ddp_like_state(r, seed=5), snap)
        for a, b in zip(states[r]["model"].state_dict().values(), fresh["model"].state_dict().values()):
            assert torch.equal(a, b)


def test_a_missing_peer_file_makes_the_step_unavailable(tmp_path):
    """A layout that points into another rank's file is only offered when that file is complete
    (a rank that died mid-write leaves none): the step is not restored from half a snapshot."""
    world = 2
    states = [_ddp_like_state(r) for r in range(world)]
    rescues, jobs = _group_take(tmp_path, world, states)
    owner = max(range(world), key=lambda r: jobs[r]["bytes"])
    os.unlink(tmp_path / f"rank{owner}-step7.bin")
    assert all(rescues[r].available(1, world) == [] for r in range(world))


def test_digests_tell_apart_what_differs():
    from devspace_amd.rescue import digests

    x = torch.randn(300_000)
    y = x.clone()
    y[123_456] = y[123_456] + 1.0
    base = torch.randn(1001)
    d = digests([x, x.clone(), y, x.view(torch.int32), base[1:], torch.ones(3, dtype=torch.bool), torch.zeros(0, 3)])
    assert d[0] == d[1] and d[0] != d[2] and d[0] != d[3]  # same bytes, other dtype: not the same tensor
    assert d[4] == digests([base[1:].clone()])[0]  # a view at an odd offset


def test_tensors_that_differ_by_a_swap_of_two_words_each_write_their_own_copy(tmp_path):
    """a position-insensitive row checksum took two ranks' tensors that differ
    only by a swap of two 8-byte words inside a row for one tensor, wrote it once, and the other
    rank restored the wrong bytes. With the position-keyed digest each rank writes its own copy,
    and both restore bit-exact; a plain sum of the words is the same for both."""
    world = 2
    torch.manual_seed(3)
    a = torch.randint(-2**62, 2**62, (1 << 19,), dtype=torch.int64)  # 4 MiB
    b = a.clone()
    b[1000], b[1001] = a[1001].item(), a[1000].item()
    assert not torch.equal(a, b) and a.sum() == b.sum()
    floats = torch.randn(1 << 20)  # the same swap in float data (a sign flip pair)
    f2 = floats.clone()
    f2[10], f2[12] = -floats[10].abs(), floats[10].abs()
    f1 = floats.clone()
    f1[10], f1[12] = floats[10].abs(), -floats[10].abs()
    states = [{"w": a, "f": f1}, {"w": b, "f": f2}]
    rescues, jobs = _group_take(tmp_path, world, states)
    assert jobs[0]["bytes"] >= (4 << 20) + (4 << 20) and jobs[1]["bytes"] >= (4 << 20) + (4 << 20), jobs
    for r in range(world):
        snap, _ = rescues[r].load(7, torch.device("cpu"))
        assert torch.equal(snap["w"], states[r]["w"]) and torch.equal(snap["f"], states[r]["f"]), r


def test_digests_are_position_sensitive_and_agree_across_paths():
    from devspace_amd.rescue import _ROW, _digest_rows_torch, digests

    x = torch.arange(3 * _ROW + 5, dtype=torch.int64) * 7919
    y = x.clone()
    y[[4, 5]] = y[[5, 4]]
    z = x.clone()
    z[0] += 1
    z[1] -= 1  # the plain sums cannot tell
    d = digests([x, y, z])
    assert len(set(d)) == 3
    rows = _digest_rows_torch(x)
    assert rows.shape == (4, 2) and int(rows[3, 0]) == int(x[3 * _ROW:].sum())


def test_cpu_digest_of_the_extension_matches_the_torch_path():
    """CPU-resident state goes through the extension's one-pass `state_digest_cpu` when the
    extension is loaded (8 ranks digesting 2 GiB each with a dozen torch ops per chunk took 16 s
    on the GPU box's CPUs); the numbers are the torch path's, bit for bit."""
    from devspace_amd.rescue import _ROW, _digest_kernel, _digest_rows_torch

    e = _digest_kernel(build=False)
    if e is None:
        pytest.skip("fused-ops extension not importable here")
    torch.manual_seed(4)
    ts = [torch.randint(-2**62, 2**62, (n,), dtype=torch.int64) for n in (1, 7, _ROW, 3 * _ROW + 11, 0)]
    want = torch.cat([_digest_rows_torch(t) for t in ts if t.numel()])
    assert torch.equal(e.state_digest_cpu(ts), want)


@pytest.mark.gpu
def test_digest_kernel_matches_the_torch_path_bit_for_bit():
    """The gfx950 `state_digest` kernel computes the same (S, M) row pairs as the CPU torch path,
    so a tensor's digest does not depend on where it lives (fp32 reference check of an integer op:
    exact equality)."""
    from devspace_amd.ops import fused
    from devspace_amd.rescue import _ROW, _digest_rows_torch, digests

    e = fused.ext()
    assert e is not None and hasattr(e, "state_digest"), "fused-ops extension with state_digest not loaded"
    torch.manual_seed(0)
    sizes = [1, 63, _ROW - 1, _ROW, _ROW + 1, 5 * _ROW + 77, 3 << 20]
    ts = [torch.randint(-2**62, 2**62, (n,), dtype=torch.int64) for n in sizes]
    got = e.state_digest([t.cuda() for t in ts]).cpu()
    want = torch.cat([_digest_rows_torch(t) for t in ts])
    assert torch.equal(got, want)
    mixed = [torch.randn(1000, 513, dtype=torch.bfloat16), torch.randn(7), torch.ones(3, dtype=torch.bool),
             torch.randn(4097, dtype=torch.float64)[1:]]
    assert digests([t.cuda() for t in mixed]) == digests(mixed)


def test_staging_budget_is_the_largest_copy_the_room_allows():
    gib = 1 << 30
    for free, reserved, peak in ((10 * gib, 4 * gib, 3 * gib), (gib, 0, 0), (0, 2 * gib, 2 * gib)):
        b = runner.Rescue.hbm_budget(free, reserved, peak)
        assert b >= 0
        if b:
            assert runner.Rescue.hbm_room(b - 16, free, reserved, peak)
            assert not runner.Rescue.hbm_room(b + (1 << 20), free, reserved, peak)


def test_staging_room_leaves_the_steps_their_peak():
    """the staged HBM copy may only use memory the next steps do not need.
    free + reserved - peak must hold the copy (plus 10 % and a margin); cached memory that the
    step's activations reuse is not room."""
    GiB = 1 << 30
    room = runner.Rescue.hbm_room
    # 200 GiB in use at peak, 20 GiB of it activations cached between steps, 60 GiB free
    assert room(40 * GiB, free=60 * GiB, reserved=200 * GiB, peak=200 * GiB)
    # the same job within one state size of the capacity: 10 GiB free, 40 GiB cached for the
    # activations -> round 4 counted the cache and staged; the next step would have run out
    assert not room(30 * GiB, free=10 * GiB, reserved=240 * GiB, peak=240 * GiB)
    # cache beyond the steps' peak (a freed earlier allocation) is room
    assert room(30 * GiB, free=10 * GiB, reserved=280 * GiB, peak=240 * GiB)
