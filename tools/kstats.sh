#!/bin/bash
# Register / LDS / spill counts of the kernels in one built object whose
# mangled name contains $2:  tools/kstats.sh head head_fwd_kernel
set -eu
o=$(dirname "$0")/../avr_amd/csrc/build/$1.hip.o
d=$(mktemp -d)
/opt/rocm/lib/llvm/bin/llvm-objcopy -O binary --only-section=.hip_fatbin "$o" "$d/fat.bin"
/opt/rocm/lib/llvm/bin/clang-offload-bundler --unbundle --type=o --input="$d/fat.bin" \
    --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output="$d/k.co"
/opt/rocm/lib/llvm/bin/llvm-readelf --notes "$d/k.co" | python3 -c '
import re, sys
pat = sys.argv[1]
for b in sys.stdin.read().split("  - .agpr_count"):
    m = re.search(r"\.name:\s+(\S+)", b)
    if not m or pat not in m.group(1): continue
    g = lambda k: (re.search(r"\.%s:\s+(\S+)" % k, b) or [None, None])[1]
    print(m.group(1)[:110], "vgpr", g("vgpr_count"), "agpr", b.split()[0] if b.split() else "?", "spill", g("vgpr_spill_count"))
' "$2"
rm -rf "$d"
