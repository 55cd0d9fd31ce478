export TMPDIR=/tmp
for pad in 0 12000 24000 44000; do
  SLAMHOT_LIB=tools/libslamhot_exp.so SLAMHOT_FAST_LDS_PAD=$pad timeout -k 10 120 python bench.py --no-cpu-baseline --match-pairs 0 --lba-windows 0 --pose-frames 0 --stereo-pairs 0 > gpurun_out/pad_$pad.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/pad_$pad.json')); print('pad=$pad', d['value'], d['ms_per_step'], d['stages_ms_per_step'])"
done
