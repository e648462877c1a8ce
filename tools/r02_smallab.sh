# A/B of calibration builds on the small configs (tools/small_configs.py) under rocprof, one box: main, then each
# diag/lib_<name>.so named on the command line (after its quant GPU tests), then main again
set -u
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/prof
export TMPDIR=/tmp
for v in main "$@" main; do
  if [ $v = main ]; then L=$PWD/fl_sim_amd/libflcodec.so; else L=$PWD/diag/lib_$v.so; fi
  if [ $v != main ]; then
    FLC_LIB=$L timeout -k 10 300 python -u -m pytest tests/test_gpu_codec.py -k "quant or dither or auto" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/sab_${v}_tests.log 2>&1 || { tail -5 gpurun_out/sab_${v}_tests.log; exit 1; }
  fi
  FLC_LIB=$L timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/sab_$v -o run --output-format csv -- python3 tools/small_configs.py > gpurun_out/sab_$v.log 2>&1 || exit $?
  python3 - $v <<'PY'
import csv, glob, sys
v = sys.argv[1]
f = glob.glob(f"gpurun_out/prof/sab_{v}/**/*kernel_stats.csv", recursive=True)[0]
lines = [l.strip() for l in open(f"gpurun_out/sab_{v}.log") if "us/step" in l]
ks = [(r["Name"].split("(")[0].replace("void flc::(anonymous namespace)::", "")[:40], round(float(r["AverageNs"]) / 1000, 2))
      for r in csv.DictReader(open(f)) if "quant" in r["Name"]]
print(v, lines, ks)
PY
done
