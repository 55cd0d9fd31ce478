export TMPDIR=/tmp
for i in 1 2; do for L in tools/libslamhot_prev.so tools/libslamhot_w1.so tools/libslamhot_w2.so; do
SLAMHOT_LIB=$L timeout -k 10 120 python bench.py --no-cpu-baseline --match-pairs 0 --lba-windows 0 --pose-frames 0 --stereo-pairs 0 > gpurun_out/ab.json 2>/dev/null || exit 1
python3 -c "import json,sys; d=json.load(open('gpurun_out/ab.json')); print(sys.argv[1], d['value'], d['stages_ms_per_step'])" $L
done; done
