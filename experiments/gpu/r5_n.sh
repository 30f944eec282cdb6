#!/bin/bash
# round 5 (n): the server burst of 4 clients (bench.py server extras) with burst coalescing (10 ms max, 3 ms
# quiet) + chunked interleaved admission (256-token chunks), coalescing only, interleaving only.
# The first pass of this recipe (chunk 64, 6 / 1.5 ms) and the scheduler GPU tests: see profiles/r5_batch
set -o pipefail
O=gpurun_out/r5_n
mkdir -p $O
export TMPDIR=/tmp
for cfg in "10 256" "10 0" "0 256"; do
  set -- $cfg
  OMX_ADMIT_COALESCE_MS=$1 OMX_ADMIT_CHUNK=$2 timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --batch-extra 0 --ttft-long 0 --long-ctx "" > $O/bench_c$1_k$2.log 2>&1 || { tail -20 $O/bench_c$1_k$2.log; exit 1; }
  echo "coalesce $1 chunk $2: $(tail -1 $O/bench_c$1_k$2.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); s=d["extra"]["server"]; print(d["value"], s["served_ttft_ms"], s["concurrent_per_client_tok_s"], s["concurrent_prompt_eval_ms"], s["concurrent_eval_ms"], s["concurrent_aggregate_tok_s"])')"
done
