# A/B timing of alternative libfcship builds under alt/ against the in-tree one.
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-ab}; mkdir -p $O
echo "base: $(timeout -k 10 300 python tools/bsw_bench.py 2>/dev/null | tail -1)" | tee -a $O/ab.log || exit 1
for f in alt/*.so; do
  echo "$f: $(FCSHIP_LIB=$PWD/$f timeout -k 10 300 python tools/bsw_bench.py 2>/dev/null | tail -1)" | tee -a $O/ab.log || exit 1
done
