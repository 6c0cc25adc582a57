#!/bin/bash
# gpurun (round 5): GPU suite, the basic tier's shading-batch A/B, the C2
# 1/8-shard A/B and a C2 bench line, each step under its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
OUT=gpurun_out/r05batch
mkdir -p $OUT
timeout -k 10 480 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 500 python3 scripts/ab.py 128 4 ${AB_VARIANTS:-base bb64 bb52 bb60 bb56i} > $OUT/ab_c2.json 2> $OUT/ab_c2.err || { echo "ab failed"; tail -5 $OUT/ab_c2.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/ab_c2.json')); [print(k, round(v['kernel_ms_min'],2), [round(x,2) for x in v['kernel_ms']], v['rmse_vs_first']) for k,v in d.items() if isinstance(v,dict) and 'kernel_ms_min' in v]"
timeout -k 10 300 python3 scripts/tail_ab.py c2 - 3 RT_TAIL_PERMILLE=500 > $OUT/tail_c2.jsonl 2> $OUT/tail_c2.err || { echo "tail failed"; tail -5 $OUT/tail_c2.err; exit 1; }
tail -1 $OUT/tail_c2.jsonl | python3 -c 'import json,sys; d=json.load(sys.stdin); [print("tail", k, round(v["full_min"],2), round(v["worst8_min"],3), round(v["eff8"],4)) for k,v in d["settings"].items()]'
timeout -k 10 300 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > $OUT/bench_c2.log 2>&1 || { echo "bench failed"; tail -5 $OUT/bench_c2.log; exit 1; }
tail -1 $OUT/bench_c2.log | python3 -c 'import json,sys; d=json.load(sys.stdin); print("bench", d["value"], d["ms_per_step"], d["roofline"]["kernel_ms_avg"])'
echo batch-done
