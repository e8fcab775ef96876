#!/bin/bash
# Disassemble the gfx950 code object of a built engine library:
#   tools/devdis.sh lib.so > lib.s     (address column stripped, for diffs)
set -eu
LLVM=/opt/rocm/lib/llvm/bin
t=$(mktemp -d)
$LLVM/llvm-objcopy --dump-section .hip_fatbin=$t/fb "$1"
$LLVM/clang-offload-bundler --unbundle --type=o --input=$t/fb \
  --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=$t/co
$LLVM/llvm-objdump -d --no-show-raw-insn $t/co | sed -E 's/^ *[0-9a-f]+://; s/ *\/\/ [0-9A-F]+:.*$//'
rm -rf $t
