#!/bin/bash
# Release artefacts, one client binary per OS/arch like the reference's cross-builds
# (/root/reference/scripts/build-all.bash:24-62). The CLI runs on the developer's machine, which
# is usually not the MI355X node: a laptop (darwin) reaches the node's cluster over the network.
#
# RELEASE_TARGETS lists "<os>-<arch>" targets (default: the host's, e.g. linux-amd64):
#   linux-*    static, stripped, the Linux platform layer (inotify, eventfd, ...)
#   darwin-*, other POSIX systems
#              -DDEVSPACE_PORTABLE=ON (POSIX platform layer, stat-scan watcher), dynamically
#              linked, cross-compiled with cmake/toolchains/<target>.cmake (an osxcross or
#              similar toolchain; none ships in this image). docs/platforms.md lists what
#              darwin and windows still need.
# A target whose toolchain file is missing fails the run: nothing is released half.
# Writes into $DIST_DIR (default dist/):
#   devspace-<os>-<arch>            the client
#   devspace-helper-linux-amd64     static, stripped in-container sync agent (runs in the pod)
#   <binary>.sha256, checksums.txt  the digests `devspace upgrade` verifies before swapping
#   latest                          the version, for a plain DEVSPACE_RELEASE_URL mirror
# RELEASE_BUILD_DIR=<dir> packages the executables of an existing static build (bin/ of the
# in-tree build) for the host target instead of configuring fresh builds.
set -euo pipefail
cd "$(dirname "$0")/.."
DIST=${DIST_DIR:-dist}

host_target() {
  local os arch
  os=$(uname -s | tr '[:upper:]' '[:lower:]')
  case "$(uname -m)" in
    x86_64|amd64) arch=amd64 ;;
    aarch64|arm64) arch=arm64 ;;
    *) arch=$(uname -m) ;;
  esac
  echo "$os-$arch"
}
HOST=$(host_target)
TARGETS=${RELEASE_TARGETS:-$HOST}

mkdir -p "$DIST"
summed=()

# package <built binary> <artefact name> <strip tool>
package() {
  local src=$1 dst=$2 strip_tool=$3
  cp "$src" "$DIST/$dst.tmp"
  "$strip_tool" --strip-all "$DIST/$dst.tmp" 2>/dev/null || "$strip_tool" "$DIST/$dst.tmp"
  chmod 0755 "$DIST/$dst.tmp"
  mv "$DIST/$dst.tmp" "$DIST/$dst"
  (cd "$DIST" && sha256sum "$dst" > "$dst.sha256")
  summed+=("$dst")
}

helper_bin=""
for t in $TARGETS; do
  os=${t%%-*}
  if [ -n "${RELEASE_BUILD_DIR:-}" ]; then
    [ "$t" = "$HOST" ] || { echo "release: RELEASE_BUILD_DIR packages the host target only ($HOST), not $t" >&2; exit 1; }
    BIN=bin
  else
    B=build-release-$t
    args=(-G Ninja -DCMAKE_BUILD_TYPE=Release -DDEVSPACE_PYTHON=OFF "-DDEVSPACE_OUTPUT_DIR=$PWD/$B/bin")
    if [ "$t" != "$HOST" ]; then
      tc=cmake/toolchains/$t.cmake
      [ -f "$tc" ] || { echo "release: no toolchain for $t ($tc)" >&2; exit 1; }
      args+=("-DCMAKE_TOOLCHAIN_FILE=$PWD/$tc")
    fi
    if [ "$os" = linux ]; then
      args+=(-DDEVSPACE_STATIC=ON)
    else
      args+=(-DDEVSPACE_PORTABLE=ON -DDEVSPACE_STATIC=OFF)
    fi
    cmake -S . -B "$B" "${args[@]}" > /dev/null
    ninja -C "$B" devspace $([ "$t" = "$HOST" ] && echo devspace-helper)
    BIN=$B/bin
  fi
  if [ "$os" = linux ] && ldd "$BIN/devspace" > /dev/null 2>&1; then
    echo "release: $BIN/devspace is dynamically linked (configure with -DDEVSPACE_STATIC=ON)" >&2
    exit 1
  fi
  strip_tool=strip
  [ "$t" = "$HOST" ] || strip_tool=${RELEASE_STRIP:-strip}
  package "$BIN/devspace" "devspace-$t" "$strip_tool"
  if [ "$t" = "$HOST" ]; then
    helper_bin=$BIN/devspace-helper
    "$BIN/devspace" version | awk '{print $3}' > "$DIST/latest"
  fi
done
# the in-container helper runs in the pod (linux-amd64 GPU nodes), whatever the client's OS
if [ -n "$helper_bin" ] && [ "$HOST" = linux-amd64 ]; then
  package "$helper_bin" devspace-helper-linux-amd64 strip
elif [ -x bin/devspace-helper ]; then
  package bin/devspace-helper devspace-helper-linux-amd64 strip
fi
(cd "$DIST" && for f in "${summed[@]}"; do cat "$f.sha256"; done > checksums.txt)
ls -l "$DIST"
