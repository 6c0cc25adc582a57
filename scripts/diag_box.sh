set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r04
AB_WORKLOAD=c4 DIAG_LIB=librt_mi355x_diag_t1.so timeout -k 10 300 python3 scripts/diag.py 16 > gpurun_out/r04/diag_c4.json 2> gpurun_out/r04/diag_c4.err || { echo diag c4 failed; tail -5 gpurun_out/r04/diag_c4.err; exit 1; }
cat gpurun_out/r04/diag_c4.json | head -30
AB_WORKLOAD=c5 DIAG_LIB=librt_mi355x_diag_t2.so timeout -k 10 300 python3 scripts/diag.py 16 > gpurun_out/r04/diag_c5.json 2> gpurun_out/r04/diag_c5.err || { echo diag c5 failed; tail -5 gpurun_out/r04/diag_c5.err; exit 1; }
cat gpurun_out/r04/diag_c5.json | head -30
AB_WORKLOAD=c2 DIAG_LIB=librt_mi355x_diag.so timeout -k 10 300 python3 scripts/diag.py 64 > gpurun_out/r04/diag_c2.json 2> gpurun_out/r04/diag_c2.err || { echo diag c2 failed; tail -5 gpurun_out/r04/diag_c2.err; exit 1; }
cat gpurun_out/r04/diag_c2.json | head -30
