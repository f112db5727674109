"""Numerics of the gfx950 fused ops (devspace_amd/ops/fused_ops.hip) against fp32 PyTorch
references of the same ops, plus the CPU fallback path of the wrappers."""
import pytest
import torch
import torch.nn.functional as F

from devspace_amd.ops import fused


def _ref_rmsnorm(x, w, eps):
    xf = x.float()
    return xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps) * w.float()


def test_cpu_fallbacks_match_torch():
    torch.manual_seed(0)
    x = torch.randn(4, 6, 32)
    w = torch.randn(32)
    assert torch.allclose(fused.rms_norm(x, w, 1e-6), F.rms_norm(x, (32,), w, 1e-6))
    h = torch.randn(5, 16)
    g, u = h.chunk(2, -1)
    assert torch.allclose(fused.swiglu(h), F.silu(g) * u)
    logits = torch.randn(7, 24)
    t = torch.randint(0, 24, (7,))
    assert torch.allclose(fused.cross_entropy(logits, t), F.cross_entropy(logits, t))
    m = fused.RMSNorm(32)
    assert m.weight.shape == (32,) and m(x).shape == x.shape


def test_extension_is_built_from_this_source(tmp_path, monkeypatch):
    """The in-tree extension carries the SHA-256 of the fused_ops.hip it was compiled from, and
    loading one built from other source bytes is an error (stale kernels never run quietly)."""
    try:
        from devspace_amd.ops import _fused_ops
    except ImportError as e:
        pytest.skip(f"extension not built here: {e}")
    from devspace_amd.ops import build

    assert _fused_ops.source_sha == build.source_sha()
    edited = tmp_path / "fused_ops.hip"
    edited.write_bytes(open(build.os.path.join(build.HERE, "fused_ops.hip"), "rb").read() + b"// edit\n")
    monkeypatch.setattr(build, "source_sha", lambda path=None: _sha(edited))
    with pytest.raises(RuntimeError, match="stale"):
        fused._check_source(_fused_ops)


def _sha(path):
    import hashlib

    return hashlib.sha256(open(path, "rb").read()).hexdigest()


gpu = pytest.mark.gpu


@gpu
def test_gpu_runs_kernels_built_from_this_source():
    dev = _cuda()
    print(f"fused_ops.hip sha256 {fused.check_fresh()[:16]} == the loaded extension's")
    x = torch.randn(64, 256, device=dev, dtype=torch.bfloat16)
    w = torch.randn(256, device=dev, dtype=torch.bfloat16)
    ref = _ref_rmsnorm(x, w, 1e-6)
    assert torch.allclose(fused.rms_norm(x, w, 1e-6, kernel=True).float(), ref, atol=3e-2, rtol=3e-2)


def _cuda():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    fused.ext()  # the HIP extension must load on a GPU box (no eager fallback)
    return torch.device("cuda")


@gpu
@pytest.mark.parametrize("rows,dim", [(4096, 1024), (37, 768), (8, 4096), (5, 24)])
def test_rmsnorm_fwd_bwd(rows, dim):
    dev = _cuda()
    torch.manual_seed(1)
    x = torch.randn(rows, dim, device=dev).bfloat16().requires_grad_()
    w = (1 + 0.1 * torch.randn(dim, device=dev)).bfloat16().requires_grad_()
    eps = torch.finfo(torch.bfloat16).eps
    y = fused.rms_norm(x, w, eps, kernel=True)  # the gfx950 kernel (the default path is PyTorch's)
    dy = torch.randn_like(y)
    y.backward(dy)
    xr = x.detach().float().requires_grad_()
    wr = w.detach().float().requires_grad_()
    yr = _ref_rmsnorm(xr, wr, eps)
    yr.backward(dy.float())
    torch.testing.assert_close(y.float(), yr, atol=2e-2, rtol=2e-2)
    torch.testing.assert_close(x.grad.float(), xr.grad, atol=3e-2, rtol=3e-2)
    # weight grad sums over all rows: compare relative to its scale
    err = (w.grad.float() - wr.grad).abs().max() / wr.grad.abs().max()
    assert err < 2e-2, err


@gpu
@pytest.mark.parametrize("rows,hidden", [(4096, 2730), (64, 1024), (3, 6)])
def test_swiglu_fwd_bwd(rows, hidden):
    dev = _cuda()
    torch.manual_seed(2)
    h = torch.randn(rows, 2 * hidden, device=dev).bfloat16().requires_grad_()
    y = fused.swiglu(h)
    dy = torch.randn_like(y)
    y.backward(dy)
    hr = h.detach().float().requires_grad_()
    g, u = hr.chunk(2, -1)
    yr = F.silu(g) * u
    yr.backward(dy.float())
    torch.testing.assert_close(y.float(), yr, atol=2e-2, rtol=2e-2)
    torch.testing.assert_close(h.grad.float(), hr.grad, atol=2e-2, rtol=2e-2)


@gpu
@pytest.mark.parametrize("rows,vocab,ignore", [(4096, 8192, False), (33, 1000, True), (2, 32000, False)])
def test_cross_entropy_fwd_bwd(rows, vocab, ignore):
    dev = _cuda()
    torch.manual_seed(3)
    logits = (3 * torch.randn(rows, vocab, device=dev)).bfloat16().requires_grad_()
    t = torch.randint(0, vocab, (rows,), device=dev)
    if ignore:
        t[::4] = -100
    loss = fused.cross_entropy(logits, t)
    loss.backward()
    lr = logits.detach().float().requires_grad_()
    ref = F.cross_entropy(lr, t, ignore_index=-100)
    ref.backward()
    torch.testing.assert_close(loss.float(), ref, atol=1e-4, rtol=1e-4)
    n = (t != -100).sum().item()  # compare per-row gradients at O(1) scale
    torch.testing.assert_close(logits.grad.float() * n, lr.grad * n, atol=2e-3, rtol=2e-2)


def _ref_attention(qkv, causal):
    q, k, v = qkv.float().unbind(2)
    o = F.scaled_dot_product_attention(q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2), is_causal=causal)
    return o.transpose(1, 2)


def test_attention_cpu_fallback_matches_sdpa():
    torch.manual_seed(5)
    qkv = torch.randn(2, 16, 3, 2, 8)
    torch.testing.assert_close(fused.attention(qkv, causal=True), _ref_attention(qkv, True))


@gpu
@pytest.mark.parametrize("b,t,h,causal", [(2, 256, 3, True), (2, 256, 3, False), (8, 512, 16, True), (1, 1024, 2, True)])
def test_attention_fwd_bwd(b, t, h, causal):
    dev = _cuda()
    torch.manual_seed(6)
    qkv = torch.randn(b, t, 3, h, 64, device=dev).bfloat16().requires_grad_()
    assert fused.ext().attention_supported(qkv)
    o = fused.attention(qkv, causal=causal)
    assert o.shape == (b, t, h, 64) and o.is_contiguous()
    do = torch.randn_like(o)
    o.backward(do)
    qr = qkv.detach().float().requires_grad_()
    orf = _ref_attention(qr, causal)
    orf.backward(do.float())
    torch.testing.assert_close(o.float(), orf, atol=2e-2, rtol=2e-2)
    for i, name in enumerate("qkv"):
        g, gr = qkv.grad[:, :, i].float(), qr.grad[:, :, i]
        err = (g - gr).abs().max() / gr.abs().max()
        assert err < 3e-2, (name, float(err))


def _adamw_pair(dev, dtype):
    torch.manual_seed(4)
    shapes = [(300, 64), (1024,), (7, 3), (8192, 16)]
    ps = [torch.randn(s, device=dev).to(dtype) for s in shapes]
    a = [p.clone().requires_grad_() for p in ps]
    b = [p.clone().requires_grad_() for p in ps]
    return a, b


def test_adamw_cpu_matches_torch():
    a, b = _adamw_pair(torch.device("cpu"), torch.float32)
    oa = fused.AdamW(a, lr=1e-2, weight_decay=0.1)
    ob = torch.optim.AdamW(b, lr=1e-2, weight_decay=0.1)
    for it in range(3):
        for x, y in zip(a, b):
            g = torch.randn_like(x)
            x.grad, y.grad = g.clone(), g.clone()
        oa.step()
        ob.step()
    for x, y in zip(a, b):
        torch.testing.assert_close(x, y, atol=1e-6, rtol=1e-5)


@gpu
def test_adamw_hip_matches_torch_fused():
    dev = _cuda()
    a, b = _adamw_pair(dev, torch.bfloat16)
    oa = fused.AdamW(a, lr=1e-2, weight_decay=0.1)
    ob = torch.optim.AdamW(b, lr=1e-2, weight_decay=0.1, fused=True)
    for it in range(5):
        for x, y in zip(a, b):
            g = torch.randn_like(x)
            x.grad, y.grad = g.clone(), g.clone()
        oa.step()
        ob.step()
    for x, y in zip(a, b):
        # both keep bf16 params/moments with fp32 math: equal up to a bf16 ulp now and then
        torch.testing.assert_close(x.float(), y.float(), atol=2e-2, rtol=2e-2)
        assert (x.float() - y.float()).abs().mean() < 2e-3
    assert all(oa.state[x]["step"] == 5 for x in a)


@gpu
def test_tinylm_step_uses_fused_ops_and_trains():
    """The rocm-pytorch example's model built on the fused ops: loss goes down over steps."""
    import importlib.util
    import os

    dev = _cuda()
    path = os.path.join(os.path.dirname(__file__), "..", "examples", "rocm-pytorch", "train.py")
    spec = importlib.util.spec_from_file_location("tinylm_train", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    assert mod.RMSNorm is fused.RMSNorm and mod.swiglu is fused.swiglu
    mod.LAYERS, mod.SEQ, mod.BATCH = 2, 128, 4

    class Ctx:
        rank, distributed, device = 0, False, dev

        def preempt_point(self):  # runner.Context hook; nothing to preempt here
            pass

        def log(self, msg):
            print(msg)

    state = mod.setup(Ctx())
    losses = [mod.step(Ctx(), state)["loss"] for _ in range(8)]
    assert losses[-1] < losses[0], losses


def test_gemm_tuning_modes_cpu():
    from devspace_amd.ops import gemm_tuning

    assert gemm_tuning.apply("off")["active"] is False
    # no GPU here: every mode reports inactive instead of touching TunableOp
    assert gemm_tuning.apply("shipped")["active"] is (torch.cuda.is_available() and torch.version.hip is not None
                                                     and gemm_tuning._arch(0) == "gfx950")
    with pytest.raises(ValueError):
        gemm_tuning.apply("sometimes")
    assert gemm_tuning._count(gemm_tuning.SHIPPED) > 0


@gpu
def test_gemm_tuning_shipped_table_loads_on_gfx950():
    _cuda()
    from devspace_amd.ops import gemm_tuning

    if gemm_tuning._arch(0) != "gfx950":
        pytest.skip("table is for gfx950")
    rep = gemm_tuning.apply("shipped")
    try:
        assert rep["active"] and rep["entries"] >= 10
        a = torch.randn(4096, 1024, device="cuda").bfloat16()
        b = torch.randn(1024, 3072, device="cuda").bfloat16()
        torch.testing.assert_close((a @ b).float(), a.float() @ b.float(), atol=0.5, rtol=2e-2)
    finally:
        torch.cuda.tunable.enable(False)


def test_add_rms_norm_cpu_fallback():
    torch.manual_seed(7)
    x, d, w = torch.randn(3, 5, 32), torch.randn(3, 5, 32), torch.randn(32)
    s, y = fused.add_rms_norm(x, d, w, 1e-6)
    torch.testing.assert_close(s, x + d)
    torch.testing.assert_close(y, F.rms_norm(x + d, (32,), w, 1e-6))


@gpu
@pytest.mark.parametrize("rows,dim,use_ds", [(4096, 1024, True), (37, 768, True), (64, 1024, False)])
def test_add_rms_norm_fwd_bwd(rows, dim, use_ds):
    dev = _cuda()
    torch.manual_seed(8)
    x = torch.randn(rows, dim, device=dev).bfloat16().requires_grad_()
    d = torch.randn(rows, dim, device=dev).bfloat16().requires_grad_()
    w = (1 + 0.1 * torch.randn(dim, device=dev)).bfloat16().requires_grad_()
    eps = torch.finfo(torch.bfloat16).eps
    s, y = fused.add_rms_norm(x, d, w, eps)
    dy, ds = torch.randn_like(y), torch.randn_like(s)
    (((y.float() * dy.float()).sum() + (s.float() * ds.float()).sum()) if use_ds else (y.float() * dy.float()).sum()).backward()
    xr, dr, wr = (t.detach().float().requires_grad_() for t in (x, d, w))
    sr = (xr + dr).bfloat16().float()  # the fused kernel rounds s to bf16 like the eager add
    yr = _ref_rmsnorm(sr, wr, eps)
    loss = (yr * dy.float()).sum() + ((sr * ds.float()).sum() if use_ds else 0)
    loss.backward()
    torch.testing.assert_close(s.float(), (x.float() + d.float()), atol=2e-2, rtol=1e-2)
    torch.testing.assert_close(y.float(), yr, atol=2e-2, rtol=2e-2)
    torch.testing.assert_close(x.grad.float(), xr.grad, atol=3e-2, rtol=3e-2)
    torch.testing.assert_close(d.grad.float(), dr.grad, atol=3e-2, rtol=3e-2)
    err = (w.grad.float() - wr.grad).abs().max() / wr.grad.abs().max()
    assert err < 2e-2, err
