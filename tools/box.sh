#!/bin/bash
# On the GPU box (via gpurun), from the repo root: the steps of one call, in order, each under a
# time limit of its own, stopping at the first failure (a GPU step that faults, aborts or times
# out ends the call: nothing more runs on the GPU after it).
#
#   tools/box.sh <tag> <step> [<step> ...]
#
# Steps (outputs under gpurun_out/<tag>/):
#   suite                the whole GPU suite (pytest -m gpu)
#   suite=<sel>[,<sel>]  pytest on the given files / node ids (comma-separated), -m gpu
#   smoke                __graft_entry__.smoke()
#   bench                the driver's default line (config 3: --steps 20 --warmup 5)
#   bench=N,chains,iters,steps   a short bench line of that shape (no CPU baseline)
#   ab=<variants>        tools/box_abn.sh over $MH_AB_CFGS ("main" = the product library,
#                        others abvar/libmhgpu_<v>.so), $MH_AB_REPS alternations
#   prof=N,chains,iters,steps    tools/profile_box.sh: kernel trace + the PMC passes
#   bound                tools/bound_check.py (every room, full length)
#   bound=<room>,N,chains,steps,kernel[;...]   those cases only
#   stamps=N,chains,iters        tools/stamps.py on abvar/libmhgpu_stamps.so
#   spread=N,chains,launches,iters  tools/launch_spread.py (per-launch time and bound decisions)
# Example:
#   gpurun --timeout 1200 -- 'bash tools/box.sh r06a suite smoke bench=64,65536,1000,3'
set -o pipefail
TAG=${1:?tag}; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$TAG; mkdir -p "$OUT"

line() {  # the bench line's headline fields
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('%s value=%.4g ms/launch=%.3f mean=%.10g acc=%d e2e=%s' % (sys.argv[2], d['value'], d['kernel_ms_per_launch'], d['mean_final_cost'], d['accepted'], d.get('e2e_chain_steps_per_s')))" "$1" "$2"
}

for STEP in "$@"; do
  KEY=${STEP%%=*}; VAL=${STEP#*=}; [ "$VAL" = "$STEP" ] && VAL=""
  NAME=$(echo "$STEP" | tr '=,/:' '____' | cut -c1-60)
  case $KEY in
    suite)
      SEL=${VAL//,/ }; SEL=${SEL:-tests}
      timeout -k 10 1000 python -u -m pytest $SEL -m gpu -x -v --timeout 300 --timeout-method thread \
          -p no:cacheprovider -W always::UserWarning > "$OUT/$NAME.log" 2>&1
      rc=$?; grep -E "ParityReport|passed|failed|Error|violat" "$OUT/$NAME.log" | tail -40
      [ $rc -eq 0 ] || { tail -30 "$OUT/$NAME.log"; exit $rc; } ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.txt" 2>&1 \
          || { tail -20 "$OUT/smoke.txt"; exit 1; }
      tail -2 "$OUT/smoke.txt" ;;
    bench)
      if [ -z "$VAL" ]; then
        timeout -k 10 400 python bench.py --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err" \
            || { tail -5 "$OUT/bench.err"; exit 1; }
        line "$OUT/bench.json" default
      else
        set -- ${VAL//,/ }
        timeout -k 10 300 python bench.py --objects $1 --chains $2 --iters $3 --steps $4 --warmup 1 \
            --no-cpu-baseline > "$OUT/$NAME.json" 2> "$OUT/$NAME.err" || { tail -5 "$OUT/$NAME.err"; exit 1; }
        line "$OUT/$NAME.json" "N=$1"
      fi ;;
    ab)
      bash tools/box_abn.sh "$TAG/ab" ${VAL//,/ } || exit 1 ;;
    prof)
      set -- ${VAL//,/ }
      bash tools/profile_box.sh "$TAG/prof_n$1" --objects $1 --chains $2 --iters $3 --steps $4 \
          --warmup 1 --no-cpu-baseline --e2e-iters 0 || exit 1 ;;
    bound)  # (bound=<room>,N,chains,steps,kernel[;...]: those cases only)
      if [ -z "$VAL" ]; then
        timeout -k 10 1000 python -u tools/bound_check.py > "$OUT/bound.txt" 2>&1
      else
        for CASE in ${VAL//;/ }; do
          timeout -k 10 300 python -u tools/bound_check.py --one ${CASE//,/ } >> "$OUT/bound.txt" 2>&1 || break
        done
      fi
      rc=$?; grep "\[bound\]" "$OUT/bound.txt"; [ $rc -eq 0 ] || { tail -20 "$OUT/bound.txt"; exit $rc; } ;;
    stamps)
      set -- ${VAL//,/ }
      MH_LIB=abvar/libmhgpu_stamps.so timeout -k 10 300 python tools/stamps.py $1 $2 $3 \
          > "$OUT/stamps_n$1.txt" 2>&1 || { tail -10 "$OUT/stamps_n$1.txt"; exit 1; }
      tail -25 "$OUT/stamps_n$1.txt" ;;
    spread)  # tools/launch_spread.py: per-launch time beside the check build's decision counts
      set -- ${VAL//,/ }
      timeout -k 10 600 python tools/launch_spread.py $1 $2 $3 $4 > "$OUT/spread_n$1.txt" 2>&1 \
          || { tail -20 "$OUT/spread_n$1.txt"; exit 1; }
      cat "$OUT/spread_n$1.txt" ;;
    *) echo "box.sh: unknown step '$STEP'"; exit 2 ;;
  esac
done
echo "box.sh $TAG: done"
