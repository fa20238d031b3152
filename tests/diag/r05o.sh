# Round 5: extremum kernel segment lengths -- time (kernel trace) and FETCH_SIZE per 128 x 1080p
# extract for the shipped build and variants (tests/build_variant.sh), GPU box.
set -o pipefail
OUT=gpurun_out/r05o
mkdir -p $OUT
export TMPDIR=/tmp
for cfg in base:X=0 ew64:SGPU_LIB_PATH=build_exp/ew64/libsiftgpu.so ew48:SGPU_LIB_PATH=build_exp/ew48/libsiftgpu.so base2:X=0 ew64b:SGPU_LIB_PATH=build_exp/ew64/libsiftgpu.so; do
  name=${cfg%%:*}; envs=${cfg#*:}
  env $envs timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $OUT/kt_$name -o run -- python3 tests/probe.py extract --reps 3 > $OUT/kt_$name.log 2>&1 || exit 1
  env $envs timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_$name -o run -- python3 tests/probe.py extract --reps 2 > $OUT/pmc_$name.log 2>&1 || exit 1
  python3 - $OUT $name <<'PY'
import csv, sys, statistics, glob
out, name = sys.argv[1], sys.argv[2]
kt = list(csv.DictReader(open(glob.glob(f"{out}/kt_{name}/**/*kernel_trace.csv", recursive=True)[0])))
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in kt if "k_extrema" in r["Kernel_Name"]]
pm = [r for r in csv.DictReader(open(glob.glob(f"{out}/pmc_{name}/**/*counter_collection.csv", recursive=True)[0])) if "k_extrema" in r["Kernel_Name"]]
f = [float(r["Counter_Value"]) * 1024 * 2 / 1e9 for r in pm]
print(f"{name}: extrema {statistics.median(d[-3:]):.1f} us, FETCH x2 {statistics.median(f):.3f} GB (alg 8.460)")
PY
done
