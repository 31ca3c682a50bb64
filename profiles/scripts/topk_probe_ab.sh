set -o pipefail
BLP_LIB=$PWD/bipartite-link-prediction_amd/blp/libblp_tkprof.so timeout -k 10 300 python profiles/scripts/topk_probe.py && bash profiles/scripts/ab_topk.sh
