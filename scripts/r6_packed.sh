#!/bin/bash
# GPU session (scripts/r6_packed.sh TAG): the streamed-result tests (values and EL_STREAM_PACKED),
# then G3 and G3E with the packed stream against the 4-byte value stream, alternating, three
# rounds: wall, init / saturate / copy-back split and the bytes that crossed PCIe.  VARIANTS
# (env, e.g. "lib:ocol") adds variant libraries, run with the value stream.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "stream or digest or export" > $OUT/t.log 2>&1
rc=$?; tail -2 $OUT/t.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" $OUT/t.log | head -20; exit $rc; }
for w in g3 g3e; do
  B="bench.py --no-cpu --no-profile --no-throughput2 --steps 10 --warmup 3 --workload $w"
  timeout -k 10 200 python $B > $OUT/warm_$w.json 2> $OUT/warm_$w.err || { tail $OUT/warm_$w.err; exit 1; }
  for rep in 1 2 3; do
    for c in packed stream ${VARIANTS}; do
      E=""; F="--copyback $c"
      case "$c" in lib:*) E="EL_LIB_VARIANT=${c#lib:}"; F="--copyback stream"; c=${c#lib:} ;; esac
      env $E timeout -k 10 200 python $B $F > $OUT/${w}_${c}_$rep.json 2> $OUT/${w}_${c}_$rep.err || { tail $OUT/${w}_${c}_$rep.err; exit 1; }
      echo "$w $c $rep $(python -c "import json; d=json.load(open('$OUT/${w}_${c}_$rep.json')); print(d['ms_per_step'], d['init_ms'], d['saturate_ms'], d['copyback_ms'], d['copyback_bytes'])")"
    done
  done
done
