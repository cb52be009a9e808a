#!/bin/bash
# Build libvrhip.so variants for scripts/ab.py: each argument is NAME=FLAGS,
# e.g.  bash scripts/build_variants.sh base= w5="-DVR_PATH_BLOCK=256 -DVR_PATH_WAVES=5"
# Writes $VDIR/libvrhip_NAME.so and $VDIR/NAME.log (VDIR: abl/, which travels to
# the GPU box for A/B runs -- delete it afterwards; variants/ is kept off the box) (kernel resource
# usage remarks of every translation unit); prints the C2 path kernel's
# VGPRs / spills.  Variants build one after another (each build is parallel).
set -e
cd "$(dirname "$0")/.."
VDIR=${VDIR:-abl}
mkdir -p $VDIR
for spec in "$@"; do
  name=${spec%%=*}; flags=${spec#*=}
  rm -f $VDIR/libvrhip_$name.so
  python3 - "$name" "$flags" "$VDIR" > $VDIR/$name.log 2>&1 <<'PY' || { grep -m5 error: $VDIR/$name.log; echo "$name: BUILD FAILED"; continue; }
import shlex, sys
sys.path.insert(0, ".")
from vrenderer_pathtracer_amd import build
name, flags, vdir = sys.argv[1], sys.argv[2], sys.argv[3]
build.build(force=True, verbose=True, out_path=f"{vdir}/libvrhip_{name}.so",
            extra_flags=shlex.split(flags) + ["-Rpass-analysis=kernel-resource-usage"])
PY
  grep -E -A12 "render_wave_kernelILi16ELj2147483657ELi[0-9]+E" $VDIR/$name.log | grep -E "VGPRs:|VGPRs Spill|Scratch" \
    | sed 's/.*remark: *//;s/ \[-Rpass.*//' | tr '\n' ' ' | sed "s/^/$name: /"; echo
done
