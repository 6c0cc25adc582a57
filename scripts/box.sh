#!/bin/bash
# One gpurun call, any sequence of steps (replaces the per-round r0N_*_box.sh):
#   gpurun -- 'OUT=r06a STEPS="tests bench" bash scripts/box.sh'
# Steps (STEPS, run in order):
#   tests       the GPU suite (TESTS, default "tests -m gpu")
#   checktests  the same on the bounds-checked build (librt_mi355x_check.so)
#   bench       bench.py BENCH_ARGS for each workload in BENCH_WORKLOADS (default c2)
#   ab          interleaved A/B (scripts/ab.py AB_SPP AB_REPS AB_VARIANTS) on each of AB_WORKLOADS
#   diag        diagnostic builds, one per "workload:lib:spp" in DIAG_RUNS (scripts/diag.py)
#   ffp         whole-frame parity (scripts/full_frame_parity.py) for each of FFP (C5 at FFP_C5_SPP)
#   density     VALU exec density (one --pmc pass) of each A/B variant in DENS_VARIANTS on DENS_WORKLOADS
#   tail        1/8-shard rehearsal (scripts/tail_ab.py) for each of TAIL_WORKLOADS
# Output under gpurun_out/$OUT.  Every GPU step has its own time limit; a
# fault / abort / kill / timeout status (124, 134, 137, 139) or any failure
# ends the call (steps are never retried).
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-box}
mkdir -p $O
stop() { echo "FAILED: $1 (status $2)"; exit $2; }
for step in ${STEPS:-tests}; do
  case $step in
    tests)
      timeout -k 10 ${TEST_TIMEOUT:-600} python3 -u -m pytest ${TESTS:-tests -m gpu} -x -q -s --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
      rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || { tail -40 $O/pytest.log; stop tests $rc; } ;;
    checktests)
      RT_MI355X_LIB=raytracer-2025_amd/librt_mi355x_check.so timeout -k 10 ${TEST_TIMEOUT:-600} python3 -u -m pytest ${TESTS:-tests -m gpu} -x -q -s --timeout 120 --timeout-method thread > $O/pytest_check.log 2>&1
      rc=$?; tail -3 $O/pytest_check.log; [ $rc -eq 0 ] || { tail -40 $O/pytest_check.log; stop checktests $rc; } ;;
    bench)
      for w in ${BENCH_WORKLOADS:-c2}; do
        timeout -k 10 ${BENCH_TIMEOUT:-600} python3 bench.py --workload $w ${BENCH_ARGS:-} > $O/bench_$w.json 2> $O/bench_$w.err
        rc=$?; [ $rc -eq 0 ] || { tail -5 $O/bench_$w.err; stop "bench $w" $rc; }
        python3 -c "import json; d=json.load(open('$O/bench_$w.json')); r=d['roofline']; cb=d.get('cpu_baseline') or {}; print('bench $w', d['value'], d['ms_per_step'], r['kernel_ms_avg'], r['frac'], cb.get('speedup_whole_host'))"
      done ;;
    ab)
      for w in ${AB_WORKLOADS:-c2}; do
        AB_WORKLOAD=$w timeout -k 10 ${AB_TIMEOUT:-500} python3 scripts/ab.py ${AB_SPP:-128} ${AB_REPS:-3} ${AB_VARIANTS:-base} > $O/ab_$w.json 2> $O/ab_$w.err
        rc=$?; [ $rc -eq 0 ] || { tail -5 $O/ab_$w.err; stop "ab $w" $rc; }
        python3 -c "import json; d=json.load(open('$O/ab_$w.json')); [print('$w', k, round(v['kernel_ms_min'],2), [round(x,2) for x in v['kernel_ms']], v['rmse_vs_first']) for k,v in d.items() if isinstance(v,dict) and 'kernel_ms_min' in v]"
      done ;;
    diag)
      for d in ${DIAG_RUNS:-c2:librt_mi355x_diag.so:64}; do
        w=${d%%:*}; rest=${d#*:}; lib=${rest%%:*}; spp=${rest##*:}
        AB_WORKLOAD=$w DIAG_LIB=$lib timeout -k 10 300 python3 scripts/diag.py $spp > $O/diag_$w.json 2> $O/diag_$w.err
        rc=$?; [ $rc -eq 0 ] || { tail -5 $O/diag_$w.err; stop "diag $w" $rc; }
        python3 -c "import json; d=json.load(open('$O/diag_$w.json')); d.pop('raw', None); print('diag $w', d)"
      done ;;
    ffp)
      for w in ${FFP:-c2 c3}; do
        spp=""; [ "$w" = c5 ] && spp=${FFP_C5_SPP:-64}
        timeout -k 10 ${FFP_TIMEOUT:-600} python3 -u scripts/full_frame_parity.py $w $spp > $O/ffp_$w.jsonl 2> $O/ffp_$w.err
        rc=$?; [ $rc -eq 0 ] || { tail -5 $O/ffp_$w.err; stop "ffp $w" $rc; }
        tail -1 $O/ffp_$w.jsonl
      done ;;
    density)
      # VALU exec density of A/B variants: one --pmc pass per (workload, variant)
      for w in ${DENS_WORKLOADS:-c5}; do
        for v in ${DENS_VARIANTS:-base}; do
          RT_MI355X_LIB=raytracer-2025_amd/librt_ab_$v.so timeout -k 10 300 timeout -s KILL 290 rocprofv3 --pmc SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES --output-format csv -d $O/dens_${w}_$v -o run -- python3 bench.py --workload $w --steps 1 --warmup 1 --spp ${DENS_SPP:-64} --no-cpu-baseline --no-host-rate > $O/dens_${w}_$v.log 2>&1
          rc=$?; [ $rc -eq 0 ] || { tail -5 $O/dens_${w}_$v.log; stop "density $w $v" $rc; }
          python3 scripts/exec_density.py $O/dens_${w}_$v/run_counter_collection.csv $w $v | tee $O/dens_${w}_$v.json
        done
      done ;;
    tail)
      for w in ${TAIL_WORKLOADS:-c2}; do
        TAIL_WARM=1 timeout -k 10 300 python3 scripts/tail_ab.py $w - 3 > $O/tail_$w.jsonl 2> $O/tail_$w.err
        rc=$?; [ $rc -eq 0 ] || { tail -5 $O/tail_$w.err; stop "tail $w" $rc; }
        tail -1 $O/tail_$w.jsonl
      done ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo box-done
