# SW lane/pair kernel occupancy statistics from the diagnostic build alt/stats.so
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-sws}; mkdir -p $O
FCSHIP_LIB=$PWD/alt/stats.so timeout -k 10 300 python tools/bsw_stats.py --reads 250000 > $O/stats.log 2>&1; rc=$?
grep -v amdgpu.ids $O/stats.log | tail -60
exit $rc
