export TMPDIR=/tmp
for L in prev new; do
SLAMHOT_LIB=tools/libslamhot_$L.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rp_$L -o run -- python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 --batch 32 --match-pairs 0 --pose-frames 0 --stereo-pairs 0 --lba-calls 6 > /dev/null 2>&1 || exit 1
python3 - <<PY
import csv,glob
f=glob.glob("gpurun_out/rp_$L/**/run_kernel_stats.csv", recursive=True)[0] if glob.glob("gpurun_out/rp_$L/**/run_kernel_stats.csv", recursive=True) else "gpurun_out/rp_$L/run_kernel_stats.csv"
for r in csv.DictReader(open(f)):
    if "lba::" in r["Name"]: print("$L", r["Name"].split("(")[0], r["Calls"], round(float(r["AverageNs"])/1000,1))
PY
done
