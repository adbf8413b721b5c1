#!/bin/bash
# Register / LDS / spill counts of the kernels in one .hip source (device-only
# compile for gfx950, read from the code object's metadata notes).
#   bash tools/kernel_resources.sh csrc/ctc_beam_v32.hip [kernel-name-regex]
set -eu
R=$(cd "$(dirname "$0")/.." && pwd)
P=$R/gpu-accelerated-speech-recognition_amd
T=$(mktemp -d)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -mcode-object-version=5 -O3 -std=c++17 -ffp-contract=off \
    -I$R/include -I$P/csrc ${KR_FLAGS:-} --cuda-device-only -c "$P/$1" -o $T/b.co
/opt/rocm/lib/llvm/bin/clang-offload-bundler --unbundle --type=o --input=$T/b.co \
    --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=$T/d.o
/opt/rocm/lib/llvm/bin/llvm-readelf --notes $T/d.o | \
    grep -E "^\s+\.name:|\.vgpr_count|\.sgpr_count|spill_count|\.private_segment_fixed_size" | \
    paste - - - - - - | grep -E "${2:-.}" | sed 's/  */ /g'
rm -rf $T
