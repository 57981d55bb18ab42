#!/bin/bash
# One parametrised entry point for the GPU-box measurements (run through gpurun from the repo
# root). Every GPU step runs under its own time limit and the steps are chained with `set -e`,
# so a failure ends the call. Outputs go under gpurun_out/ (copy what is to be kept into
# profiles/<round>/).
#
#   bash scripts/gpu.sh tests [pytest args...]        GPU suite (default: all of tests/ -m gpu)
#   bash scripts/gpu.sh bench [bench.py args...]      one bench line -> gpurun_out/bench.json
#   bash scripts/gpu.sh round ROUND [BATCH]           the round bundle: rocprofv3 --stats of the
#        bench, FETCH_SIZE / WRITE_SIZE passes -> profiles/ROUND/traffic.json, the
#        rocprof-vs-HIP-event agreement table, then the default bench line
#   bash scripts/gpu.sh ab-env VAR "v1 v2 ..." [REPS]  interleaved bench A/B of an env switch
#   bash scripts/gpu.sh ab-lib "main base ..." [REPS] [STEPS]  interleaved bench A/B of library
#        builds (scripts/build_variant.sh REV NAME -> dna_amd/lib/libdna_amd_NAME.so)
#   bash scripts/gpu.sh stats OUT -- CMD...           rocprofv3 --kernel-trace --stats of CMD
#   bash scripts/gpu.sh pmc OUT [KERNEL_RE] -- CMD... SQ counter sets + FETCH_SIZE + WRITE_SIZE,
#        one rocprofv3 --pmc pass each (kernel-trace only, never combined with other traces),
#        summarised by scripts/pmc_table.py
# (The per-session gpu_r*/gpu_s* recipes of rounds 1-3 were folded into this script; git history
# keeps them.)
set -e
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
mkdir -p gpurun_out
cmd=$1
shift || true

case "$cmd" in
tests)
  args=("$@")
  [ ${#args[@]} -eq 0 ] && args=(tests/)
  timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
    -p no:cacheprovider "${args[@]}" > gpurun_out/gpu_tests.log 2>&1
  tail -3 gpurun_out/gpu_tests.log
  ;;
bench)
  timeout -k 10 600 python bench.py "$@" > gpurun_out/bench.json 2> gpurun_out/bench.err
  cat gpurun_out/bench.json
  ;;
round)
  R=${1:?round}
  BATCH=${2:-512}
  OUT=$ROOT/gpurun_out/$R
  mkdir -p "$OUT" "$ROOT/profiles/$R"
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/stats -o run --output-format csv -- \
    python $ROOT/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-b64 --batch $BATCH \
    > $OUT/stats_bench.json 2> $OUT/stats_bench.err
  for c in FETCH_SIZE WRITE_SIZE; do
    d=$(echo $c | cut -d_ -f1 | tr A-Z a-z)
    timeout -k 10 600 rocprofv3 --kernel-trace --pmc $c -d $OUT/$d -o run --output-format csv -- \
      python $ROOT/bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-b64 --no-data-pipeline \
      --batch $BATCH > $OUT/${d}_bench.json 2> $OUT/${d}_bench.err
  done
  python $ROOT/scripts/traffic_from_pmc.py $OUT/fetch $OUT/write $OUT/traffic.json $BATCH \
    $OUT/fetch_bench.json > /dev/null
  cp $OUT/traffic.json $ROOT/profiles/$R/traffic.json
  python $ROOT/scripts/prof_summary.py $OUT/stats/run_kernel_stats.csv --steps 13 > $OUT/kernel_stats.md
  python $ROOT/scripts/roofline_agree.py $OUT/stats/run_kernel_stats.csv $OUT/stats_bench.json 13 \
    > $OUT/roofline_agreement.md
  cd $ROOT
  timeout -k 10 600 python bench.py --batch $BATCH > $OUT/bench.json 2> $OUT/bench.err
  rm -rf $OUT/fetch $OUT/write
  ;;
ab-env)
  VAR=${1:?var}
  VALS=${2:?values}
  REPS=${3:-2}
  for rep in $(seq $REPS); do
    for v in $VALS; do
      env $VAR=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline \
        --no-b64 --no-data-pipeline > gpurun_out/ab.json 2> gpurun_out/ab.err
      echo "$VAR=$v $(python -c "import json;d=json.load(open('gpurun_out/ab.json'));print(d['value'], d['ms_per_step'], {k: round(v['avg_ms'],3) for k,v in d['kernels'].items()})")"
    done
  done | tee gpurun_out/ab.log
  ;;
ab-lib)
  # interleaved bench A/B of library builds (scripts/build_variant.sh): LIBS = "main base ..."
  # names libdna_amd.so ("main") or dna_amd/lib/libdna_amd_<name>.so
  LIBS=${1:?libs}
  REPS=${2:-2}
  STEPS=${3:-20}
  for rep in $(seq $REPS); do
    for l in $LIBS; do
      if [ "$l" = main ]; then f=$ROOT/dna_amd/lib/libdna_amd.so; else f=$ROOT/dna_amd/lib/libdna_amd_$l.so; fi
      DNA_AMD_LIB=$f timeout -k 10 300 python bench.py --steps $STEPS --warmup 5 --no-cpu-baseline \
        --no-b64 --no-data-pipeline > gpurun_out/ab.json 2> gpurun_out/ab.err
      echo "$l $(python -c "import json;d=json.load(open('gpurun_out/ab.json'));print(d['value'], d['ms_per_step'], {k: round(v['avg_ms'],3) for k,v in d['kernels'].items()})")"
    done
  done | tee gpurun_out/ab.log
  ;;
ab-tree)
  # interleaved bench A/B of whole source trees (scripts/build_tree_variant.sh REV NAME ->
  # _ab/NAME): TREES = "main base ..." ("main" = this tree)
  TREES=${1:?trees}
  REPS=${2:-2}
  STEPS=${3:-20}
  for rep in $(seq $REPS); do
    for t in $TREES; do
      if [ "$t" = main ]; then b=$ROOT/bench.py; else b=$ROOT/_ab/$t/bench.py; fi
      timeout -k 10 300 python $b --steps $STEPS --warmup 5 --no-cpu-baseline \
        --no-b64 --no-data-pipeline > gpurun_out/ab.json 2> gpurun_out/ab.err
      echo "$t $(python -c "import json;d=json.load(open('gpurun_out/ab.json'));print(d['value'], d['ms_per_step'], {k: round(v['avg_ms'],3) for k,v in d['kernels'].items()})")"
    done
  done | tee gpurun_out/ab.log
  ;;
fftpmc)
  # config-D FFT long conv: rocprofv3 --stats + separate FETCH_SIZE / WRITE_SIZE passes of
  # scripts/fftconv_bench.py, per-kernel traffic table (scripts/fft_traffic.py) -> $OUT/traffic.md
  OUT=$ROOT/gpurun_out/${1:?out}
  shift
  mkdir -p $OUT
  cd /tmp && export TMPDIR=/tmp
  ARGS="--B 2 --D 256 --L 65536 --dtype bf16 --bidirectional 1 --iters 5"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- \
    python $ROOT/scripts/fftconv_bench.py $ARGS > $OUT/bench.txt 2>&1
  for c in FETCH_SIZE WRITE_SIZE; do
    d=$(echo $c | cut -d_ -f1 | tr A-Z a-z)
    timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $OUT/$d -o run -- \
      python $ROOT/scripts/fftconv_bench.py $ARGS > $OUT/$d.log 2>&1
  done
  python $ROOT/scripts/fft_traffic.py $OUT/fetch $OUT/write $OUT/stats/run_kernel_stats.csv > $OUT/traffic.md
  cat $OUT/bench.txt $OUT/traffic.md
  rm -rf $OUT/fetch $OUT/write
  ;;
stats)
  OUT=$ROOT/gpurun_out/${1:?out}
  shift
  [ "$1" = "--" ] && shift
  mkdir -p $OUT
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- "$@" \
    > $OUT/cmd.log 2>&1
  python $ROOT/scripts/prof_summary.py $OUT/run_kernel_stats.csv > $OUT/kernel_stats.md || true
  ;;
pmc)
  OUT=$ROOT/gpurun_out/${1:?out}
  shift
  KRE="."
  if [ "$1" != "--" ]; then KRE=$1; shift; fi
  [ "$1" = "--" ] && shift
  mkdir -p $OUT
  cd /tmp && export TMPDIR=/tmp
  i=0
  for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_MFMA" \
             "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE" \
             "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC" \
             "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    timeout -s KILL 180 rocprofv3 --kernel-trace --pmc $set -d $OUT/set_$i -o run --output-format csv \
      -- "$@" > $OUT/set_$i.log 2>&1
  done
  python $ROOT/scripts/pmc_table.py $OUT --kernel "$KRE" > $OUT/summary.txt 2>&1 || true
  python $ROOT/scripts/pmc_table.py $OUT --kernel "$KRE" --per-kernel > $OUT/per_kernel.txt 2>&1 || true
  cat $OUT/per_kernel.txt
  ;;
*)
  sed -n 2,20p "$0"
  exit 2
  ;;
esac
