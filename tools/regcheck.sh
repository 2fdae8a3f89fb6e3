#!/bin/bash
# Register / spill report of every kernel in libfsagg.so (gfx950 code
# objects): name, vgpr_count, sgpr_spill_count, vgpr_spill_count, scratch.
set -e
d=$(mktemp -d)
cp "$(dirname "$0")/../federatedscope_amd/lib/libfsagg.so" "$d/lib.so"
cd "$d"
/opt/rocm/lib/llvm/bin/llvm-objdump --offloading lib.so > /dev/null
for co in lib.so.*gfx950*; do
  /opt/rocm/lib/llvm/bin/llvm-readelf --notes "$co"
done | python3 -c "
import sys, re
cur = {}
rows = []
for line in sys.stdin:
    m = re.match(r'\s+\.(name|vgpr_count|sgpr_spill_count|vgpr_spill_count|private_segment_fixed_size|agpr_count):\s+(\S+)', line)
    if not m: continue
    k, v = m.groups()
    if k == 'name':
        cur = {'name': v}; rows.append(cur)
    else:
        cur[k] = int(v)
for r in rows:
    print(r.get('vgpr_count', 0), r.get('agpr_count', 0), r.get('sgpr_spill_count', 0), r.get('vgpr_spill_count', 0), r.get('private_segment_fixed_size', 0), r['name'])
"
rm -rf "$d"
