#!/bin/bash
# tools/gpu.sh STEP [STEP ...] -- the GPU-box steps of this repo, one script
# instead of one-off files.  Every GPU step runs under its own time limit; the
# chain stops at the first failure (exit status of that step).  Output goes to
# gpurun_out/$TAG/ (TAG defaults to "run").
#
#   tests                 pytest -m gpu, the whole suite (-x, per-test timeout)
#   tests:EXPR            pytest -m gpu -k EXPR
#   smoke                 __graft_entry__.smoke()
#   bench[:CFG[:ARGS]]    the driver's bench command (--steps 20 --warmup 5),
#                         config CFG (1500 default); ARGS: extra bench.py flags,
#                         '+' for spaces (e.g. bench:1500:--submit+launch)
#   bench400[:CFG]        400 steps, no side legs
#   prof[:CFG]            rocprofv3 --kernel-trace --stats of 400 steps with HIP
#                         launches (the profiler serializes the AQL engine's
#                         queues) + tools/prof_summary.py
#   pmc:CFG:C1,C2,..      one rocprofv3 --pmc pass (counters only, 20 steps)
#   py:SCRIPT[:ARGS]      python tools/SCRIPT with ARGS ('+' for spaces), stdout
#                         to $O/SCRIPT.jsonl
#   pmcpy:SCRIPT:C1,C2,..[:ARGS]  one rocprofv3 --pmc pass over python tools/SCRIPT
#   host                  the box's identity (hostname, GPU serial, driver, clocks)
#   rehearse2             the driver's N = 2 bench command, two ranks on device 0 over gloo
#   rehearse:N            the same with N ranks (N <= 8)
#
#   /usr/local/graft/bin/gpurun --timeout 900 -- 'TAG=r03x bash tools/gpu.sh tests smoke bench bench:9000'
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-run}
mkdir -p "$O"

fail() { echo "!! step '$1' failed (exit $2)"; exit "$2"; }

for step in "$@"; do
  IFS=: read -r kind a b c <<< "$step"
  extra=${b//+/ }
  echo "== $step ($(date +%T))"
  case $kind in
    tests)
      sel=(); [ -n "$a" ] && sel=(-k "$a")
      timeout -k 10 700 python -u -m pytest tests -m gpu -x -v -s --timeout 180 --timeout-method thread "${sel[@]}" \
        > "$O/gpu_tests${a:+_$a}.log" 2>&1 || fail "$step" $?
      tail -1 "$O/gpu_tests${a:+_$a}.log" ;;
    smoke)
      timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || fail "$step" $?
      tail -1 "$O/smoke.log" ;;
    bench)
      cfg=${a:-1500}
      sfx=$(echo "$extra" | tr -c 'A-Za-z0-9\n' '_' | sed 's/^_*//')  # one file per (config, flags)
      bj="$O/bench_$cfg${sfx:+_$sfx}"
      timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --config "$cfg" $extra \
        > "$bj.json" 2> "$bj.err" || fail "$step" $?
      cut -c1-400 "$bj.json" ;;
    bench400)
      cfg=${a:-1500}
      timeout -k 10 300 python -u bench.py --gpus 1 --steps 400 --warmup 5 --config "$cfg" --also none \
        --sustain-seconds 0 --cpu-seconds 0 --no-host-path --no-dropin $extra \
        > "$O/bench400_$cfg.json" 2>> "$O/bench400.err" || fail "$step" $?
      cut -c1-300 "$O/bench400_$cfg.json" ;;
    prof)
      cfg=${a:-1500}
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_$cfg" -o run --output-format csv -- \
        python3 bench.py --steps 400 --warmup 5 --config "$cfg" --submit launch --also none --sustain-seconds 0 \
        --cpu-seconds 0 --no-host-path --no-dropin > "$O/prof_$cfg.json" 2> "$O/prof_$cfg.err" || fail "$step" $?
      f=$(ls "$O"/prof_"$cfg"/*/run_kernel_trace.csv "$O"/prof_"$cfg"/run_kernel_trace.csv 2>/dev/null | head -1)
      kopt=(); [ "$cfg" = tx ] && kopt=(--kernel "${PROF_KERNEL:-k_tx_copy}")
      python tools/prof_summary.py "$f" "${kopt[@]}" > "$O/prof_summary_$cfg.json" || fail "$step" $?
      cut -c1-400 "$O/prof_summary_$cfg.json" ;;
    pmc)
      cfg=${a:-1500}
      tag=$(echo "$b" | tr ',' '_' | cut -c1-40)
      timeout -s KILL 120 rocprofv3 --pmc ${b//,/ } -d "$O/pmc_${cfg}_$tag" -o run --output-format csv -- \
        python3 bench.py --steps 20 --warmup 5 --config "$cfg" --submit launch --also none --sustain-seconds 0 \
        --settle 0 --warm-regions 0 --cpu-seconds 0 --no-host-path --no-dropin \
        > "$O/pmc_${cfg}_$tag.json" 2> "$O/pmc_${cfg}_$tag.err" || fail "$step" $?
      echo "pmc $cfg $b done" ;;
    py)
      scr=${a%.py}
      timeout -k 10 600 python -u "tools/$scr.py" $extra > "$O/$scr.jsonl" 2> "$O/$scr.err" || fail "$step" $?
      tail -3 "$O/$scr.jsonl" | cut -c1-300 ;;
    pmcpy)
      scr=${a%.py}
      tag=$(echo "$b" | tr ',' '_' | cut -c1-60)
      timeout -s KILL 180 rocprofv3 --pmc ${b//,/ } -d "$O/pmc_${scr}_$tag" -o run --output-format csv -- \
        python3 "tools/$scr.py" ${c//+/ } > "$O/pmc_${scr}_$tag.out" 2> "$O/pmc_${scr}_$tag.err" || fail "$step" $?
      echo "pmc $scr $b done" ;;
    rehearse2|rehearse)
      # the driver's N-rank command (rehearse2: N = 2; rehearse:N), all ranks
      # on device 0 over gloo (RCCL refuses two ranks on one device):
      # bench.py's N > 1 path end to end
      nr=2; [ "$kind" = rehearse ] && nr=${a:-2}
      MI_BENCH_DEVICE=0 MI_BENCH_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 \
        --nproc-per-node "$nr" --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus "$nr" --steps 20 --warmup 5 \
        --cpu-seconds 0 --no-host-path --no-dropin --sustain-seconds 0 $extra \
        > "$O/bench_n${nr}_rehearsal.json" 2> "$O/bench_n${nr}_rehearsal.err" || fail "$step" $?
      tail -c 400 "$O/bench_n${nr}_rehearsal.json" ;;
    host)
      { hostname; cat /sys/class/drm/card*/device/serial_number 2>/dev/null | head -8; rocm-smi --showproductname \
        --showserial --showmeminfo vram 2>/dev/null | grep -v "^$" | head -30; } > "$O/host.txt" 2>&1 || true
      head -3 "$O/host.txt" ;;
    *)
      echo "unknown step $step"; exit 2 ;;
  esac
done
echo "== all steps done ($(date +%T))"
