"""Autograd wrappers around the gfx950 fused ops (fused_ops.hip).

    from devspace_amd.ops import fused
    norm = fused.RMSNorm(dim)             # drop-in for nn.RMSNorm
    x, h = fused.add_rms_norm(x, delta, norm.weight)  # x += delta; h = norm(x), one kernel
    y = fused.swiglu(h)                   # silu(h[..., :H]) * h[..., H:]
    loss = fused.cross_entropy(logits, t) # mean CE on bf16 logits [N, V]

On a GPU the HIP kernels are mandatory: if the in-tree extension is missing or broken the
first call raises (no silent eager fallback). On CPU tensors (tests, CPU smoke runs) the plain
PyTorch formulation is used.
"""

from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

_ext = None
_ext_error = None


def _load_cached():
    """A copy of this package vendored into a project (`devspace init`, rocm-pytorch) has no
    in-tree build: compile into the cache (done at image build by the template's Dockerfile,
    else once on the first pod start) and load it from there."""
    import importlib.util

    from . import build

    path = build.ensure_fused_cached()
    spec = importlib.util.spec_from_file_location(f"{__package__}._fused_ops", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def ext():
    """The compiled extension module (raises with the build error on a GPU box)."""
    global _ext, _ext_error
    if _ext is None and _ext_error is None:
        try:
            from . import _fused_ops  # noqa: WPS433 - the in-tree (or image-built) extension

            _check_source(_fused_ops)  # a stale build raises here, on every call
            _ext = _fused_ops
        except ImportError as e:  # pragma: no cover - depends on the build
            try:
                _ext = _load_cached()
            except Exception as e2:  # no hipcc / ROCm headers in the image, build error
                _ext_error = f"{e}; building it failed: {e2}"
    if _ext is None:
        raise RuntimeError(f"devspace_amd fused HIP ops are not built ({_ext_error}); run "
                           "`python -m devspace_amd.ops.build --fused`")
    return _ext


def _check_source(mod) -> None:
    """An in-tree build must come from the source next to it: kernels older than an edit of
    fused_ops.hip must not run (an error, not a silent fallback)."""
    import os

    from . import build

    if os.path.exists(os.path.join(build.HERE, "fused_ops.hip")):
        built, src = getattr(mod, "source_sha", "unknown"), build.source_sha()
        if built != src:
            raise RuntimeError(f"the fused-ops extension is stale: built from source {built[:12]}, the source is "
                               f"{src[:12]}; run `python -m devspace_amd.ops.build --fused`")


def check_fresh() -> str:
    """The loaded extension was built from the fused_ops.hip next to it: returns the source
    SHA-256, raises on a stale build (kernels older than the source)."""
    from . import build

    _check_source(ext())
    return build.source_sha()


def backend() -> str:
    """"hip" when the gfx950 kernels are loaded (loading or compiling them now), else
    "eager (<why>)". For the training script's start-up line: never a silent fallback."""
    if not torch.cuda.is_available():
        return "eager (no GPU)"
    try:
        ext()
        return "hip"
    except RuntimeError as e:
        return f"eager ({e})"


def _use_hip(t: torch.Tensor) -> bool:
    return t.is_cuda and t.dtype == torch.bfloat16


# ------------------------------------------------------------------------------ ops
# The differentiable entry points are C++ autograd nodes inside the extension (no Python on
# the forward/backward path of the training step).


def _rmsnorm_kernel_default() -> bool:
    import os

    return os.environ.get("DEVSPACE_FUSED_RMSNORM", "1") != "0"


def rms_norm(x: torch.Tensor, weight: torch.Tensor, eps: float | None = None, kernel: bool | None = None) -> torch.Tensor:
    """RMSNorm alone: the gfx950 kernel by default (`kernel=False` or DEVSPACE_FUSED_RMSNORM=0 for
    PyTorch's fused rms_norm). Fwd+bwd on [4096x1024] it takes 25.2 us of device time against
    41.4 us (1.64x, replayed from a HIP graph); issued one call at a time from Python, both are
    bound by the host's dispatch (39.4 vs 40.6 us, 1.03x; round 5 measured 0.97x that way and
    kept it off). profiles/r6_fused_ops_ab_graph.txt. In a training step the device clock is the
    one that counts: the step is queued ahead of the GPU."""
    if eps is None:
        eps = torch.finfo(x.dtype).eps
    use = _rmsnorm_kernel_default() if kernel is None else kernel
    if use and _use_hip(x) and weight.dtype == torch.bfloat16 and ext().rmsnorm_supported(x.shape[-1]):
        return ext().rms_norm(x, weight, float(eps))
    return F.rms_norm(x, (x.shape[-1],), weight, eps)


def add_rms_norm(x: torch.Tensor, delta: torch.Tensor, weight: torch.Tensor, eps: float | None = None):
    """Residual add fused into the following RMSNorm: returns (s, y) with s = x + delta and
    y = rms_norm(s) * weight. On the GPU one kernel each way (no separate add kernel forward,
    no gradient-accumulation add backward)."""
    if eps is None:
        eps = torch.finfo(x.dtype).eps
    if (_use_hip(x) and delta.dtype == torch.bfloat16 and weight.dtype == torch.bfloat16 and delta.shape == x.shape
            and ext().rmsnorm_supported(x.shape[-1])):
        s, y = ext().add_rms_norm(x, delta, weight, float(eps))
        return s, y
    s = x + delta
    return s, F.rms_norm(s, (s.shape[-1],), weight, eps)


class RMSNorm(nn.Module):
    """nn.RMSNorm(dim) with the fused HIP forward/backward (same parameters, same eps default)."""

    def __init__(self, dim: int, eps: float | None = None):
        super().__init__()
        self.eps = eps
        self.weight = nn.Parameter(torch.ones(dim))

    def forward(self, x):
        return rms_norm(x, self.weight, self.eps)


def swiglu(h: torch.Tensor) -> torch.Tensor:
    """silu(g) * u for h = cat([g, u], -1) (the gate/up projection output)."""
    if _use_hip(h) and h.shape[-1] % 4 == 0:
        return ext().swiglu(h)
    g, u = h.chunk(2, dim=-1)
    return F.silu(g) * u


def cross_entropy(logits: torch.Tensor, target: torch.Tensor, ignore_index: int = -100) -> torch.Tensor:
    """Mean cross-entropy of [N, V] logits (computed in fp32 from bf16 logits, no fp32 copy)."""
    if _use_hip(logits) and logits.dim() == 2 and logits.shape[1] % 8 == 0 and target.dtype == torch.long:
        return ext().cross_entropy(logits, target, int(ignore_index))
    return F.cross_entropy(logits.float(), target, ignore_index=ignore_index)


def attention(qkv: torch.Tensor, causal: bool = True, scale: float | None = None) -> torch.Tensor:
    """Multi-head attention on the packed projection output qkv [B, T, 3, H, D] -> [B, T, H, D].

    HIP flash attention (MFMA, fwd + bwd) for bf16, D == 64, T % 128 == 0; otherwise
    F.scaled_dot_product_attention on transposed views."""
    b, t, three, h, d = qkv.shape
    if three != 3:
        raise ValueError("qkv must be [B, T, 3, H, D]")
    if scale is None:
        scale = d ** -0.5
    if _use_hip(qkv) and ext().attention_supported(qkv):
        return ext().attention(qkv, bool(causal), float(scale))
    q, k, v = qkv.unbind(2)
    o = F.scaled_dot_product_attention(q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2), is_causal=causal,
                                       scale=scale)
    return o.transpose(1, 2)


# ------------------------------------------------------------------------------ AdamW


def _hip_ok(t: torch.Tensor) -> bool:
    return _use_hip(t) and t.is_contiguous() and t.data_ptr() % 16 == 0


class AdamW(torch.optim.Optimizer):
    """torch.optim.AdamW (decoupled weight decay, no amsgrad) with a multi-tensor HIP update for
    bf16 GPU parameters: one launch per <= 48 tensors, moments kept in the parameter dtype like
    torch's fused AdamW. Other parameters (CPU, fp32, non-contiguous) take the same math in
    plain PyTorch ops."""

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2):
        if lr < 0 or eps < 0 or not (0.0 <= betas[0] < 1.0 and 0.0 <= betas[1] < 1.0):
            raise ValueError("invalid AdamW hyper-parameters")
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for group in self.param_groups:
            lr, (b1, b2), eps, wd = group["lr"], group["betas"], group["eps"], group["weight_decay"]
            buckets = {}  # step -> lists for one multi-tensor launch
            for p in group["params"]:
                if p.grad is None:
                    continue
                if p.grad.is_sparse:
                    raise RuntimeError("AdamW does not support sparse gradients")
                st = self.state[p]
                if not st:
                    st["step"] = 0
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                st["step"] += 1
                g = p.grad
                if all(_hip_ok(t) for t in (p, g, st["exp_avg"], st["exp_avg_sq"])):
                    b = buckets.setdefault(st["step"], ([], [], [], []))
                    for lst, t in zip(b, (p, g, st["exp_avg"], st["exp_avg_sq"])):
                        lst.append(t)
                else:
                    _adamw_eager(p, g, st["exp_avg"], st["exp_avg_sq"], lr, b1, b2, eps, wd, st["step"])
            for step, (ps, gs, ms, vs) in buckets.items():
                ext().adamw_step(ps, gs, ms, vs, lr, b1, b2, eps, wd, step)
        return loss


def _adamw_eager(p, g, m, v, lr, b1, b2, eps, wd, step):
    pf, gf = p.float(), g.float()
    mf = m.float().mul_(b1).add_(gf, alpha=1 - b1)
    vf = v.float().mul_(b2).addcmul_(gf, gf, value=1 - b2)
    pf.mul_(1 - lr * wd)
    denom = vf.sqrt().div_((1 - b2 ** step) ** 0.5).add_(eps)
    pf.addcdiv_(mf, denom, value=-lr / (1 - b1 ** step))
    p.copy_(pf)
    m.copy_(mf)
    v.copy_(vf)
