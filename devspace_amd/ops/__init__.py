"""gfx950 HIP kernels used by the tool: the pod GPU probe (gpuprobe.hip)."""
