#!/bin/bash
# Device-only gfx950 assembly of the library and per-kernel resource use
# (VGPRs, SGPRs, spills, LDS) plus static instruction counts by class, for
# the kernels matching $1 (default k_cnet_defer).  CPU only.
cd "$(dirname "$0")/.." || exit 1
pat=${1:-k_cnet_defer}
out=${TMPDIR:-/tmp}/cndp_isa.s
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 --cuda-device-only -S -Wno-unused-parameter $EXTRA \
    -Wno-unused-result -Wno-unused-value -Iinclude -Icndp_amd/csrc cndp_amd/csrc/cndp_gpu.hip -o "$out" || exit 1
python3 - "$out" "$pat" <<'PY'
import re, sys, collections
src, pat = sys.argv[1], sys.argv[2]
txt = open(src).read().split("\n")
cur = None
cnt = collections.defaultdict(collections.Counter)
meta = {}
for l in txt:
    m = re.match(r"^(_Z\S+):\s*(;.*)?$", l)
    if m:
        cur = m.group(1)
        continue
    if cur and pat in cur:
        t = l.strip().split()
        if t and re.match(r"^[sv]_|^ds_|^global_|^buffer_|^flat_|^scratch_", t[0]):
            op = t[0]
            c = ("v" if op.startswith("v_") else "s" if op.startswith("s_") else "ds" if op.startswith("ds_")
                 else "scratch" if op.startswith("scratch_") else "mem")
            cnt[cur][c] += 1
            if op.startswith(("v_writelane", "v_readlane")):
                cnt[cur]["lane_spill"] += 1
    m = re.match(r"\s+\.(vgpr_count|sgpr_count|sgpr_spill_count|vgpr_spill_count|group_segment_fixed_size):\s+(\d+)", l)
    if m and cur:
        meta.setdefault(cur, {})[m.group(1)] = int(m.group(2))
for k in sorted(cnt):
    print(k[:60], dict(cnt[k]))
for l in txt:
    pass
PY
grep -A 30 "\.name:.*$pat" "$out" | grep -E "\.name:|vgpr_count|sgpr_count|spill|group_segment_fixed" | head -40
