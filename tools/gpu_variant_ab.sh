# Interleaved headline A/B of experiment builds (tools/build_variant.sh NAME FLAGS [FILE]):
#   tools/gpu_variant_ab.sh STAGE NAME... ("default" = the tree's library, "env:VAR=VALUE" = the tree's
#   library under that environment variable); prints value, ms per step and the isolated stage ms per
#   step of STAGE ("all": every stage) for each run, in order.
export TMPDIR=/tmp
mkdir -p gpurun_out
STAGE=$1; shift
for v in "$@"; do
  lib=orb-slam3-noted_amd/lib/libslamhot.so; envset=""; tag=$v
  case "$v" in
    default) ;;
    env:*) envset=${v#env:}; tag=$(echo "$envset" | tr '=' '_') ;;
    *) lib=orb-slam3-noted_amd/lib/ab/libslamhot_$v.so ;;
  esac
  env $envset SLAMHOT_LIB=$lib timeout -k 10 200 python3 bench.py --legs headline --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/var_$tag.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/var_$tag.json')); print('$v', d['value'], d['ms_per_step'], (lambda st: st if '$STAGE' == 'all' else st.get('$STAGE'))(d['headline_detail']['stage_ms_per_step']))"
done
