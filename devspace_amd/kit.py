"""The workload kit: the part of devspace_amd that runs inside a GPU pod (hot-reload runner +
gfx950 fused training ops), vendored into rocm-pytorch projects as a `devspace_amd/` package
next to train.py. The file list is devspace_amd/KIT; `devspace init` embeds the same files
(CMakeLists.txt), so the package is the only source.

    python -m devspace_amd.kit <project-dir> [--prebuilt]
"""

from __future__ import annotations

import glob
import os
import shutil
import sys

HERE = os.path.dirname(os.path.abspath(__file__))


def files() -> list:
    with open(os.path.join(HERE, "KIT")) as f:
        return [l.strip() for l in f if l.strip() and not l.startswith("#")]


def write_kit(project_dir: str, prebuilt: bool = False) -> list:
    """Writes the kit into <project_dir>/devspace_amd (only files whose bytes differ). With
    `prebuilt`, the in-tree gfx950 extension goes along (what the image build's
    `python -m devspace_amd.ops.build --fused --cache` step produces in a real image)."""
    dst_root = os.path.join(project_dir, "devspace_amd")
    written = []
    for rel in files():
        src, dst = os.path.join(HERE, rel), os.path.join(dst_root, rel)
        data = open(src, "rb").read()
        if os.path.exists(dst) and open(dst, "rb").read() == data:
            continue
        os.makedirs(os.path.dirname(dst), exist_ok=True)
        with open(dst + ".tmp", "wb") as f:
            f.write(data)
        os.replace(dst + ".tmp", dst)
        written.append(rel)
    if prebuilt:
        for so in glob.glob(os.path.join(HERE, "ops", "_fused_ops*.so")) + glob.glob(os.path.join(HERE, "ops", "libgpuprobe.so")):
            dst = os.path.join(dst_root, "ops", os.path.basename(so))
            if not os.path.exists(dst) or os.path.getmtime(dst) < os.path.getmtime(so):
                shutil.copy2(so, dst)
                written.append(os.path.relpath(dst, dst_root))
    return written


def main(argv=None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    if not argv:
        print(__doc__)
        return 2
    print("\n".join(write_kit(argv[0], prebuilt="--prebuilt" in argv)))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
