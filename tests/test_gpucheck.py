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
