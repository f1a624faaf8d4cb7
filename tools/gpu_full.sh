#!/bin/bash
# One GPU session for a round checkpoint: the whole GPU suite (no -x, so every
# failure is listed), then — only if no test hung or crashed — the default
# bench.py run.  usage: tools/gpu_full.sh TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/$1; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 180 --timeout-method thread \
  > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" "$OUT/pytest.log" | tail -15
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 900 python -u bench.py > "$OUT/bench.log" 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 4000 "$OUT/bench.log"; exit $rc
