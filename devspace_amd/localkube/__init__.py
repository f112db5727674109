"""Local single-node Kubernetes + Docker emulation used as the devspace local-pod backend."""

from .cluster import LocalCluster, detect_gpus  # noqa: F401
