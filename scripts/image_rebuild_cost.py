#!/usr/bin/env python3
"""What an edit of train.py costs the rocm-pytorch image: `devspace deploy` of
examples/rocm-pytorch on a fresh local cluster with the Dockerfile's RUN steps executed (the
fused gfx950 kernel build runs hipcc), then an edit of train.py and a second deploy. The second
build takes the kit copy and the kernel build from the layer cache, so only the project copy is
new (the Dockerfile order is tested in tests/test_e2e_image_layers.py).

  python scripts/image_rebuild_cost.py > rebuild.json

Prints one JSON object: wall-clock of both deploys and of their image builds, and whether the
second build reported "Using cache" for the kernel-build step.
"""
import json
import os
import shutil
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from devspace_amd.localkube.bench import bench_deploy

    work = tempfile.mkdtemp(prefix="devspace-rebuild-")
    try:
        r = bench_deploy(work, example="rocm-pytorch", gpus=1)
    finally:
        shutil.rmtree(work, ignore_errors=True)
    cold_build = r["cold_phases_ms"].get("image.build", 0.0)
    edit_build = r["edit_phases_ms"].get("image.build", 0.0)
    print(json.dumps({
        "example": "examples/rocm-pytorch",
        "what": "deploy with RUN executed (kernel build via hipcc), edit train.py, deploy again",
        "cold_deploy_s": round(r["cold_s"], 3),
        "cold_image_build_s": round(cold_build / 1000.0, 3),
        "edit_deploy_s": round(r["edit_s"], 3),
        "edit_image_build_s": round(edit_build / 1000.0, 3),
        "edit_reused_run_layer": r["edit_reused_run_layer"],
        "build_speedup": round(cold_build / edit_build, 1) if edit_build else None,
        "cold_phases_ms": r["cold_phases_ms"],
        "edit_phases_ms": r["edit_phases_ms"],
    }))


if __name__ == "__main__":
    main()
