#!/bin/bash
# Build the native extension of another git ref for an in-call A/B on the GPU box:
#   scripts/ab_build.sh REF NAME   ->  ab/NAME_C.so  (load it with ANA_NATIVE_LIB=ab/NAME_C.so)
# The ref must expose the same binding API as the working tree's Python code.
set -euo pipefail
ref=$1; name=$2
root=$(cd "$(dirname "$0")/.." && pwd)
src=$(mktemp -d /tmp/ab_src.XXXXXX)
trap 'rm -rf "$src"' EXIT
git -C "$root" archive "$ref" analyzer_amd | tar -x -C "$src"
(cd "$src" && python3 -m analyzer_amd.build_ext --jobs 8 > /dev/null)
mkdir -p "$root/ab"
cp "$src"/analyzer_amd/_C*.so "$root/ab/${name}_C.so"
echo "ab/${name}_C.so <- $ref"
