#!/bin/bash
# gpurun: the end-of-round checks.  STEPS (default "tests checktests"), then
# whole-frame parity (scripts/full_frame_parity.py) for each workload in FFP
# (default "c2 c3"; C5 at FFP_C5_SPP, default 64).  Every GPU step has its own
# time limit; the script stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out/fin
if [ -n "${STEPS-tests checktests}" ]; then STEPS="${STEPS-tests checktests}" bash scripts/r04_box.sh || exit 1; fi
for w in ${FFP:-c2 c3}; do
  spp=""; [ "$w" = c5 ] && spp=${FFP_C5_SPP:-64}
  timeout -k 10 ${FFP_TIMEOUT:-600} python3 -u scripts/full_frame_parity.py $w $spp > gpurun_out/fin/ffp_$w.jsonl 2> gpurun_out/fin/ffp_$w.err || { echo "ffp $w failed $?"; tail -5 gpurun_out/fin/ffp_$w.err; exit 1; }
  tail -1 gpurun_out/fin/ffp_$w.jsonl
done
echo fin-ok
