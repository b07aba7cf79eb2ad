#!/bin/bash
# Build the library of a git revision (or the working tree: "wt") into ab/lib_<name>.so
# for same-box A/B timing (scripts/ab_probe.py).   usage: scripts/ab_build.sh NAME REV|wt
set -e
NAME=$1; REV=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$ROOT/ab"
if [ "$REV" = wt ]; then
  cp "$ROOT/tts-max_amd/tts_amd/libtts_mi355x.so" "$ROOT/ab/lib_$NAME.so"
  exit 0
fi
W=$(mktemp -d /tmp/abwt.XXXX)
git -C "$ROOT" archive "$REV" tts-max_amd/csrc include | tar -x -C "$W"
mkdir -p "$W/tts-max_amd/tts_amd"
make -C "$W/tts-max_amd/csrc" -j8 >/dev/null 2>&1
cp "$W/tts-max_amd/tts_amd/libtts_mi355x.so" "$ROOT/ab/lib_$NAME.so"
rm -rf "$W"
