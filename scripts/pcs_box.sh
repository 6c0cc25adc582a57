#!/bin/bash
# gpurun: PC sampling of the path kernel (rocprofv3 --pc-sampling-*), on the
# line-table build librt_ab_pcs.so (the product's ISA, `make AB_NAMES=pcs ab`).
#   gpurun -- 'PCS_WORKLOADS="c2" bash scripts/pcs_box.sh'
# host_trap first; stochastic (gfx950) when host_trap is refused.  Each run
# under its own time limit; a fault, abort or kill ends the call.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-pcs}
mkdir -p $O
timeout -k 10 60 rocprofv3 -L > $O/list.txt 2>&1; echo "list rc=$?"
grep -i -A12 "pc.sampl" $O/list.txt | head -40
for w in ${PCS_WORKLOADS:-c2}; do
  case $w in c2) A="--spp 64";; c3) A="--spp 256";; c4) A="--spp 16";; c5) A="--spp 16 --width 1920";; esac
  B="bench.py --workload $w $A --steps 1 --warmup 1 --no-cpu-baseline --no-host-rate"
  for m in ${PCS_METHODS:-host_trap stochastic}; do
    if [ $m = host_trap ]; then U="--pc-sampling-unit time --pc-sampling-interval ${PCS_INTERVAL_US:-20}"; else U="--pc-sampling-unit cycles --pc-sampling-interval ${PCS_INTERVAL_CYC:-1048576}"; fi
    RT_MI355X_LIB=raytracer-2025_amd/librt_ab_pcs.so timeout -s KILL 240 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method $m $U --output-format csv -d $O/${w}_$m -o run -- python3 $B > $O/${w}_$m.log 2>&1
    rc=$?; echo "$w $m rc=$rc"; tail -3 $O/${w}_$m.log
    case $rc in 0) python3 scripts/pcsample_summary.py $O/${w}_$m > $O/${w}_$m.json 2> $O/${w}_$m.hdr; head -c 3000 $O/${w}_$m.json; break;;
               124|134|137|139) echo "FATAL $rc"; exit $rc;; esac
  done
done
echo pcs-done
