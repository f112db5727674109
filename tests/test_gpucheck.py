"""GPU probe (HIP kernels in devspace_amd/ops/gpuprobe.hip)."""
import pytest

pytestmark = pytest.mark.gpu


def test_probe_selftest_and_rates():
    from devspace_amd import gpucheck

    probe = gpucheck.Probe()
    assert probe.count() >= 1
    info = probe.info(0)
    assert "gfx950" in info["arch"], info
    assert info["compute_units"] == 256, info
    # exact MFMA tile vs host fp32 reference (identity A, asymmetric B)
    assert probe.selftest(0) == 0.0
    gbps = probe.hbm_gbps(0, 1 << 30, 5)
    tf = probe.mfma_tflops(0, 5000)
    assert gbps > 2000, gbps
    assert tf > 500, tf


def test_gpucheck_report():
    from devspace_amd import gpucheck

    rep = gpucheck.run(quick=True)
    assert rep["devices"] and not [p for p in rep["problems"] if "MFMA" in p]


def test_peer_probe_on_this_box():
    """The xGMI peer probe: a device is never its own peer; with several visible devices every
    ordered pair gets a copy rate (the driver's 8-GPU node; a 1-GPU box has no pairs)."""
    from devspace_amd import gpucheck

    probe = gpucheck.Probe()
    assert probe.peer_gbps(0, 0) == -1
    n = probe.count()
    pairs, problems = gpucheck.peer_check(probe, n)
    assert len(pairs) == n * (n - 1)
    for p in pairs:
        assert p["copy_gbps"] > 0, p
