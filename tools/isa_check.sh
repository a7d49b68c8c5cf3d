#!/bin/bash
# isa_check.sh OBJ... -- fail if a gfx950 code object in these HIP objects holds an
# instruction the library must not contain (JPEG decode "Compiler
# note"): v_ashr_pk_u8_i32, which the gfx950 backend once fused into sat17's
# packed clamps and which corrupted bytes 2-3 of packed words on MI355X.  The
# empty asm in ik_jpeg_idct.h sat17 prevents the fusion; this check keeps it so.
set -eo pipefail
L=/opt/rocm/lib/llvm/bin
tmp=$(mktemp -d)
trap 'rm -rf "$tmp"' EXIT
bad=0
for o in "$@"; do
    "$L/llvm-objcopy" --dump-section=.hip_fatbin="$tmp/f.bin" "$o" "$tmp/host.o"
    "$L/clang-offload-bundler" --type=o --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --input="$tmp/f.bin" \
        --output="$tmp/f.co" --unbundle
    n=$("$L/llvm-objdump" -d --mcpu=gfx950 "$tmp/f.co" | grep -c "v_ashr_pk_u8_i32" || true)
    if [ "$n" != "0" ]; then
        echo "isa_check: $o holds $n v_ashr_pk_u8_i32 (see DESIGN.md, JPEG decode compiler note)" >&2
        bad=1
    fi
done
exit $bad
