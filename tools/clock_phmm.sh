#!/bin/bash
# Effective clock of the stream kernels: GRBM_GUI_ACTIVE / 8 XCDs / kernel time,
# for the in-tree build and each alt/*.so.  usage: tools/clock_phmm.sh TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=gpurun_out/$1; mkdir -p "$O"; export TMPDIR=/tmp
run() {  # name [lib]
  local name=$1 lib=${2:-}
  FCSHIP_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-trace --stats -d "$O/$name" -o run \
    --output-format csv -- python3 tools/phmm_bench.py --steps 2 --warmup 1 > "$O/$name.log" 2>&1 || exit 1
}
run in_tree
for f in alt/*.so; do [ -e "$f" ] && run "$(basename "$f" .so)" "$PWD/$f"; done
python3 - "$O" <<'PY'
import csv, glob, os, sys, collections
for d in sorted(glob.glob(os.path.join(sys.argv[1], "*/"))):
    agg = collections.defaultdict(lambda: [0.0, 0.0, 0])
    for f in glob.glob(d + "**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "phmm3" not in r["Kernel_Name"]:
                continue
            k = r["Kernel_Name"][:40]
            a = agg[k]
            a[0] += float(r["Counter_Value"])
            a[1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) if "End_Timestamp" in r else 0
            a[2] += 1
    for k, (g, ns, n) in agg.items():
        print(os.path.basename(d.rstrip("/")), k, "dispatches", n, "GHz", round(g / 8 / ns, 3) if ns else None)
PY
