# HBM fetch bytes of conv layer 1 with the tap-major K order (in-tree library) and the channel-major taps 0,2,1 order
# (vlib/korder.so): does the variant's L2 reuse of tap 0's rows cut the traffic, and does the time follow it?
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pk_base -o run -- python3 tools/conv_bench.py 3 > gpurun_out/pk_base.log 2>&1 || { tail -5 gpurun_out/pk_base.log; exit 1; }
FDDM_HIP_LIB=vlib/korder.so timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pk_var -o run -- python3 tools/conv_bench.py 3 > gpurun_out/pk_var.log 2>&1 || { tail -5 gpurun_out/pk_var.log; exit 1; }
echo "== tap-major (in-tree)"; python3 tools/probe/pmc_korder.py gpurun_out/pk_base/run_counter_collection.csv
echo "== taps 0,2,1 per channel block (vlib/korder.so)"; python3 tools/probe/pmc_korder.py gpurun_out/pk_var/run_counter_collection.csv
