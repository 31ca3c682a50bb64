# Build experiment variants of libblp.so (timing probes only): exp_build.sh NAME -DFLAG...
set -e
cd $(dirname $0)/../bipartite-link-prediction_amd/csrc
name=$1; shift
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -shared -I../../include -w "$@" *.hip -o ../blp/libblp_$name.so
