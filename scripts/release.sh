#!/bin/bash
# Release artefacts for linux/amd64 (the reference cross-builds stripped static binaries per
# OS/arch, /root/reference/scripts/build-all.bash:24-62; this product targets x86_64 GPU nodes).
# Writes into $DIST_DIR (default dist/):
#   devspace-linux-amd64            static, stripped: runs on any x86_64 Linux, nothing to install
#   devspace-helper-linux-amd64     static, stripped in-container sync agent (bin/devspace-helper)
#   <binary>.sha256, checksums.txt  the digests `devspace upgrade` verifies before swapping
#   latest                          the version, for a plain DEVSPACE_RELEASE_URL mirror
# By default it configures a fresh Release build in build-release/; RELEASE_BUILD_DIR=<dir>
# packages the executables of an existing static build (bin/ of the in-tree build) instead.
set -euo pipefail
cd "$(dirname "$0")/.."
DIST=${DIST_DIR:-dist}
if [ -n "${RELEASE_BUILD_DIR:-}" ]; then
  BIN=bin
else
  B=build-release
  cmake -S . -B "$B" -G Ninja -DCMAKE_BUILD_TYPE=Release -DDEVSPACE_PYTHON=OFF -DDEVSPACE_STATIC=ON \
        "-DDEVSPACE_OUTPUT_DIR=$PWD/$B/bin" > /dev/null
  ninja -C "$B" devspace devspace-helper
  BIN=$B/bin
fi
if ldd "$BIN/devspace" > /dev/null 2>&1; then
  echo "release: $BIN/devspace is dynamically linked (configure with -DDEVSPACE_STATIC=ON)" >&2
  exit 1
fi
mkdir -p "$DIST"
for pair in "devspace:devspace-linux-amd64" "devspace-helper:devspace-helper-linux-amd64"; do
  src=${pair%%:*}; dst=${pair##*:}
  cp "$BIN/$src" "$DIST/$dst.tmp"
  strip --strip-all "$DIST/$dst.tmp"
  chmod 0755 "$DIST/$dst.tmp"
  mv "$DIST/$dst.tmp" "$DIST/$dst"
  (cd "$DIST" && sha256sum "$dst" > "$dst.sha256")
done
(cd "$DIST" && cat devspace-linux-amd64.sha256 devspace-helper-linux-amd64.sha256 > checksums.txt)
"$DIST/devspace-linux-amd64" version | awk '{print $3}' > "$DIST/latest"
ls -l "$DIST"
