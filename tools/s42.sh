# PairHMM A/B of alt/*.so, two rounds, 10 steps each
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/s42; mkdir -p $O
for r in 1 2; do for f in alt/*.so; do
  echo "$r $f: $(FCSHIP_LIB=$PWD/$f timeout -k 10 300 python tools/phmm_bench.py --steps 10 2>/dev/null | tail -1)" | tee -a $O/ab.log || exit 1
done; done
