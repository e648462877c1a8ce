# A/B of calibration builds on one box: the headline bench (no extras) under rocprof for main and each
# diag/lib_<name>.so named on the command line, main again at the end
set -u
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/prof
export TMPDIR=/tmp
for v in main "$@" main; do
  if [ $v = main ]; then L=$PWD/fl_sim_amd/libflcodec.so; else L=$PWD/diag/lib_$v.so; fi
  FLC_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/ab_$v -o run --output-format csv -- python3 bench.py --steps 30 --warmup 10 --skip-extra --skip-cpu > gpurun_out/ab_$v.log 2>&1 || exit $?
  python3 - $v <<'PY'
import csv, glob, json, sys
v = sys.argv[1]
f = glob.glob(f"gpurun_out/prof/ab_{v}/**/*kernel_stats.csv", recursive=True)[0]
line = [l for l in open(f"gpurun_out/ab_{v}.log") if l.startswith("{")][-1]
d = json.loads(line)
ks = [(r["Name"].split("(")[0].split("::")[-1][:28], round(float(r["AverageNs"]) / 1000, 1))
      for r in csv.DictReader(open(f)) if "flc::" in r["Name"]]
print(v, d["value"], d["ms_per_step"], ks)
PY
done
