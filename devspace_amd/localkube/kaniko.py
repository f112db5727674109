"""Kaniko executor emulation for the local cluster (`/kaniko/executor` inside build pods).

The devspace kaniko builder (src/build/image.cc build_kaniko, reference
builder/kaniko/kaniko.go:84) starts a pod from the kaniko image, uploads the build context to
/src via the sync engine's copy-to-container, then execs
`/kaniko/executor --dockerfile=/src/Dockerfile --context=dir:///src --destination=IMG ...`.
Here the same Dockerfile interpreter as the local Docker API builds the image into the local
registry, printing kaniko-style log lines.
"""

from __future__ import annotations

import argparse
import os
import sys
import time

from .dockerd import ImageStore, build_image


def _container_path(p):
    root = os.environ.get("DEVSPACE_CONTAINER_ROOT", "")
    if p.startswith("dir://"):
        p = p[len("dir://"):]
    return os.path.join(root, p.lstrip("/")) if root and p.startswith("/") else p


def main(argv=None):
    ap = argparse.ArgumentParser(prog="/kaniko/executor")
    ap.add_argument("--dockerfile", default="Dockerfile")
    ap.add_argument("--context", default="dir:///workspace")
    ap.add_argument("--destination", action="append", default=[])
    ap.add_argument("--build-arg", action="append", default=[])
    ap.add_argument("--target", default=None)
    ap.add_argument("--cache", default="false")
    ap.add_argument("--cache-repo", default="")
    ap.add_argument("--single-snapshot", action="store_true")
    ap.add_argument("--insecure", action="store_true")
    ap.add_argument("--skip-tls-verify", action="store_true")
    ap.add_argument("--no-push", action="store_true")
    args, unknown = ap.parse_known_args(argv)
    images_root = os.environ.get("DEVSPACE_LOCAL_IMAGES")
    if not images_root:
        print("error: not running inside a devspace local-cluster build pod", file=sys.stderr)
        return 1
    store = ImageStore(images_root)
    ctx = _container_path(args.context)
    dockerfile = _container_path(args.dockerfile)
    rel_df = os.path.relpath(dockerfile, ctx)
    buildargs = dict(a.split("=", 1) for a in args.build_arg if "=" in a)
    t0 = time.time()

    def log(msg):
        sys.stderr.write(f"INFO[{int(time.time() - t0):04d}] {msg}\n")
        sys.stderr.flush()

    if not args.destination:
        print("error: --destination is required", file=sys.stderr)
        return 1
    log(f"Resolved base name from {rel_df}")
    try:
        build_image(store, ctx, rel_df, args.destination[0], buildargs=buildargs, target=args.target, log=log)
    except Exception as e:  # kaniko exits 1 on build errors
        sys.stderr.write(f"error building image: {e}\n")
        return 1
    for dest in args.destination[1:]:
        store.tag(args.destination[0], dest)
    if not args.no_push:
        for dest in args.destination:
            log(f"Pushing image to {dest}")
            store.push(dest)
            log(f"Pushed image to 1 destinations")
    return 0


if __name__ == "__main__":
    sys.exit(main())
