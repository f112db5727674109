"""Local single-node Kubernetes + Docker emulation used as the devspace local-pod backend."""

from .cluster import LocalCluster, detect_gpus  # noqa: F401


def bench_deploy(workdir):
    from .bench import bench_deploy as _bd

    return _bd(workdir)
