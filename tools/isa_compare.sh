#!/bin/bash
# Compare one kernel's ISA between two versions of a HIP source (tools only).
#   bash tools/isa_compare.sh <kernel-symbol> <source-a.hip> <source-b.hip>
# Prints, per source: ISA line count, vmcnt wait histogram, MFMA count.
sym=$1; shift
for f in "$@"; do
    /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fno-fast-math -ffp-contract=off \
        -fno-gpu-flush-denormals-to-zero -S --cuda-device-only "$f" -o /tmp/isa_cmp.s 2>/dev/null || exit 1
    awk -v s="$sym:" 'index($0, s) == 1 {on = 1} on {print} on && /s_endpgm/ {exit}' /tmp/isa_cmp.s > /tmp/isa_cmp_k.s
    echo "== $f: $(wc -l < /tmp/isa_cmp_k.s) lines, $(grep -c v_mfma /tmp/isa_cmp_k.s) mfma"
    grep -o "s_waitcnt vmcnt([0-9]*)" /tmp/isa_cmp_k.s | sort | uniq -c | sort -rn | head -8
done
