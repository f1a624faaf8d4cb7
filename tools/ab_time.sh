# SW timing only (no parity) of the in-tree build and every alt/*.so, interleaved twice.
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-abt}; mkdir -p $O
for pass in 1 2; do
  echo "in-tree: $(timeout -k 10 300 python tools/bsw_bench.py 2>/dev/null | tail -1)" | tee -a $O/ab.txt || exit 1
  for f in alt/*.so; do
    echo "$f: $(FCSHIP_LIB=$PWD/$f timeout -k 10 300 python tools/bsw_bench.py 2>/dev/null | tail -1)" | tee -a $O/ab.txt || exit 1
  done
done
