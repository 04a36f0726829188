# One parameterised script for every GPU run (it replaces the per-round gpu_*.sh files):
#
#   gpurun -- bash scripts/gpu.sh <out> <step> [<step> ...]
#
# Results go to gpurun_out/<out>/. Steps run in order; each GPU step has its own time limit,
# and the first failure (fault, abort, limit) ends the run there — nothing after it touches
# the GPU. Steps:
#   tests                      pytest -m gpu, the whole suite
#   tests:<f1>,<f2>            just those test files (verbose, fail fast)
#   smoke                      __graft_entry__.smoke()
#   bench[:<workload>[:<args>]]  python bench.py --workload <workload> <args>; args use ',' for
#                              spaces (bench:q6:--steps,20), leading VAR=value args go to its
#                              environment (bench:q6:CUBIT_BENCH_PARTITION=0/8,--steps,20) — default:
#                              the driver's N = 1 line
#   profile:<workload>[:<args>]  rocprofv3 --kernel-trace --stats over that bench, then one
#                              --pmc pass each for FETCH_SIZE and WRITE_SIZE (never combined)
#   dist1                      the bench as one torchrun rank over RCCL (the N > 1 code path)
#   dist2                      two gloo ranks sharing the GPU (strong scaling rehearsal)
#   distg:<n>                  n gloo ranks sharing the GPU (n <= 4 here: the N = 8 case is the driver's)
#   self:<n>[:<args>]          plain `python bench.py --gpus n` with no launcher (bench.py starts its own
#                              n ranks), gloo, every rank on the one GPU (CUBIT_BENCH_SHARE_GPU=1)
#   apitrace[:<sf>,<tasks>]    HIP API + kernel + copy trace of examples/q6_scan (default 100 8), then
#                              scripts/api_timeline.py over runs 0..3 into $OUT/apitrace_runs.txt
#   merge                      scripts/merge_timing.py (the merge at 612 M rows, phases on stderr)
#   pipeline[:<args>]          examples/q6_scan (default 100 8) with CUBIT_SCAN_PHASES=1 (init_global's
#                              phases and each task's window waits on stderr), Q6_REPS=5; leading
#                              VAR=value args go to its environment (pipeline:CUBIT_SCAN_STAGE_MB=0,100,8;
#                              pipeline:Q6_AB=1,Q6_REPS=20,100,16; pipeline:100,8,--partitions,4)
#   trace:<cmd,args>           rocprofv3 --kernel-trace --memory-copy-trace --stats of a command
#   pmc:<counters>:<cmd,args>  one rocprofv3 --pmc pass (counters joined by '+', within one pass's
#                              limits: at most 8 SQ_, 4 TCC_, ...) over a command
#   soak[:<args>]              scripts/fuzz_soak.py (default 150 2000003 20000)
#   run:<cmd,args>             any other command (e.g. run:./scripts/smallbench,10)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/$1
shift
mkdir -p "$OUT"
PYT="python -u -m pytest -p no:cacheprovider --timeout 200 --timeout-method thread"
n=0
for step in "$@"; do
  n=$((n + 1))
  kind=${step%%:*}
  rest=${step#*:}
  [ "$rest" = "$step" ] && rest=""
  log=$OUT/$n.$kind.log
  echo "== step $n: $step" >&2
  case $kind in
    tests)
      if [ -n "$rest" ]; then
        timeout -k 10 600 $PYT -x -v ${rest//,/ } > "$log" 2>&1
      else
        timeout -k 10 1000 $PYT -m gpu -x -v tests > "$log" 2>&1
      fi ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$log" 2>&1 ;;
    bench)
      w=${rest%%:*}; a=${rest#*:}; [ "$a" = "$rest" ] && a=""
      envs=(); args=()
      for x in ${a//,/ }; do [[ $x == *=* && $x != --* ]] && envs+=("$x") || args+=("$x"); done
      if [ -n "$w" ]; then
        env "${envs[@]}" timeout -k 10 600 python bench.py --workload "$w" "${args[@]}" > "$OUT/$n.bench_$w.json" 2> "$log"
      else
        timeout -k 10 600 python bench.py > "$OUT/$n.bench.json" 2> "$log"
      fi ;;
    profile)
      w=${rest%%:*}; a=${rest#*:}; [ "$a" = "$rest" ] && a=""
      d=$OUT/prof/$w
      mkdir -p "$d"
      timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$d/kt" -o kt -- \
          python3 bench.py --workload "$w" --steps 20 --warmup 5 --no-cpu-baseline ${a//,/ } > "$d/bench_kt.log" 2>&1 &&
      timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$d/fetch" -o fetch -- \
          python3 bench.py --workload "$w" --steps 20 --warmup 5 --no-cpu-baseline ${a//,/ } > "$d/bench_fetch.log" 2>&1 &&
      timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$d/write" -o write -- \
          python3 bench.py --workload "$w" --steps 20 --warmup 5 --no-cpu-baseline ${a//,/ } > "$d/bench_write.log" 2>&1 ;;
    dist1)
      CUBIT_BENCH_DIST1=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
          --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline \
          --no-maintenance --no-zonemap-leg > "$OUT/$n.bench_dist1_rccl.json" 2> "$log" ;;
    dist2)
      CUBIT_BENCH_SHARE_GPU=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
          --master-addr 127.0.0.1 --master-port 29518 bench.py --gpus 2 --steps 10 --warmup 3 --dist-backend gloo \
          --no-cpu-baseline > "$OUT/$n.bench_dist2_gloo.json" 2> "$log" ;;
    distg)
      [ "$rest" -ge 2 ] && [ "$rest" -le 4 ] || { echo "distg: 2 to 4 ranks" >&2; exit 2; }
      CUBIT_BENCH_SHARE_GPU=1 timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node "$rest" \
          --master-addr 127.0.0.1 --master-port 29519 bench.py --gpus "$rest" --steps 10 --warmup 3 --dist-backend gloo \
          --no-cpu-baseline > "$OUT/$n.bench_dist${rest}_gloo.json" 2> "$log" ;;
    self)
      nn=${rest%%:*}; a=${rest#*:}; [ "$a" = "$rest" ] && a=""
      [ "$nn" -ge 2 ] && [ "$nn" -le 4 ] || { echo "self: 2 to 4 ranks" >&2; exit 2; }
      CUBIT_BENCH_SHARE_GPU=1 timeout -k 10 500 python bench.py --gpus "$nn" --steps 10 --warmup 3 \
          --dist-backend gloo --no-cpu-baseline ${a//,/ } > "$OUT/$n.bench_self${nn}_gloo.json" 2> "$log" ;;
    apitrace)
      a=${rest:-100,8}
      timeout -k 10 300 rocprofv3 --hip-runtime-trace --kernel-trace --memory-copy-trace --output-format csv \
          -d "$OUT/apitrace" -o q6 -- duckdb-cubit_amd/lib/q6_scan ${a//,/ } > "$log" 2>&1 &&
      for r in 0 1 2 3; do echo "== run $r"; python scripts/api_timeline.py "$OUT/apitrace" $r; done \
          > "$OUT/apitrace_runs.txt" 2>&1 ;;
    pipeline)
      envs=(); args=()
      for x in ${rest//,/ }; do [[ $x == *=* ]] && envs+=("$x") || args+=("$x"); done
      [ ${#args[@]} -eq 0 ] && args=(100 8)
      env CUBIT_SCAN_PHASES=1 Q6_REPS=5 "${envs[@]}" timeout -k 10 300 duckdb-cubit_amd/lib/q6_scan "${args[@]}" \
          > "$log" 2>&1 ;;
    trace)
      timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d "$OUT/trace$n" \
          -o tr -- ${rest//,/ } > "$log" 2>&1 ;;
    pmc)
      c=${rest%%:*}; a=${rest#*:}
      timeout -s KILL 300 rocprofv3 --pmc ${c//+/ } --output-format csv -d "$OUT/pmc$n" -o pmc -- ${a//,/ } \
          > "$log" 2>&1 ;;
    soak)
      a=${rest:-150,2000003,20000}
      timeout -k 10 400 python -u scripts/fuzz_soak.py ${a//,/ } > "$log" 2>&1 ;;
    merge)
      timeout -k 10 600 python -u scripts/merge_timing.py > "$log" 2>&1 ;;
    run)
      timeout -k 10 600 ${rest//,/ } > "$log" 2>&1 ;;
    *)
      echo "unknown step $step" >&2; exit 2 ;;
  esac
  rc=$?
  tail -3 "$log" >&2
  if [ $rc -ne 0 ]; then
    echo "== step $n ($step) failed: rc $rc" >&2
    exit $rc
  fi
done
for f in "$OUT"/*.json; do [ -f "$f" ] && { echo "== $f"; tail -1 "$f" | cut -c1-700; }; done
exit 0
