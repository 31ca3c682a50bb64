# every bench mode once after the wedge-row index (graph-creation cost included in the wall time)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_similarity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/sim_tests.log 2>&1 || exit 1; echo "wall $SECONDS s" >> gpurun_out/walls.txt
rm -f gpurun_out/walls.txt
SECONDS=0; timeout -k 10 300 python bench.py > gpurun_out/m_sim.json 2> gpurun_out/m_sim.err || exit 1; echo "wall $SECONDS s" >> gpurun_out/walls.txt
SECONDS=0; timeout -k 10 300 python bench.py --mode topk --no-cpu-baseline > gpurun_out/m_topk.json 2> gpurun_out/m_topk.err || exit 1; echo "wall $SECONDS s" >> gpurun_out/walls.txt
SECONDS=0; timeout -k 10 600 python bench.py --mode sharded --config c5 --no-cpu-baseline > gpurun_out/m_c5.json 2> gpurun_out/m_c5.err || exit 1; echo "wall $SECONDS s" >> gpurun_out/walls.txt
