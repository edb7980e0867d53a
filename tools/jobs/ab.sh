# A/B of library builds (tools/ab_build.sh -> ab/<name>/libmsv_hip.so) on the bench configs,
# interleaved in one call:   gpurun -- 'CONFIGS="cfg3 cfg5" REPS=2 bash tools/jobs/ab.sh base new ...'
set -e
CONFIGS=${CONFIGS:-"cfg3 cfg5 cfg2"}
REPS=${REPS:-2}
STEPS=${STEPS:-20}
mkdir -p gpurun_out/ab
for r in $(seq $REPS); do
  for c in $CONFIGS; do
    for n in "$@"; do
      MSV_LIB_PATH=$PWD/ab/$n/libmsv_hip.so timeout -k 10 240 python bench.py --no-cpu --config $c --steps $STEPS \
        > gpurun_out/ab/${n}_${c}_$r.json 2> gpurun_out/ab/${n}_${c}_$r.err
      python -c "import json;d=json.load(open('gpurun_out/ab/${n}_${c}_$r.json'));print('$n $c $r', d['kernel_ms'], d['value'])"
    done
  done
done
