# same-box A/B of environment switches: bench rounds with each "NAME=VALUE" (or "base") in turn, repeated.
# usage: bash scripts/gpu_ab_env.sh "DG_NO_FUSED_POOL=1" ...   (EXTRA: more bench flags)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
B="python bench.py --steps 30 --warmup 8 --no-cpu-baseline $EXTRA"
for r in 1 2; do
  for v in base "$@"; do
    tag=$(echo "$v" | tr -c 'A-Za-z0-9_\n' '_')
    if [ "$v" = base ]; then envs=""; else envs="$v"; fi
    env $envs timeout -k 10 300 $B > gpurun_out/ab_${tag}_$r.json 2> gpurun_out/ab_${tag}_$r.err || exit 1
    echo "$v $r $(python -c "import json;d=json.loads(open('gpurun_out/ab_${tag}_$r.json').read().strip().splitlines()[-1]);print(d['value'],(d.get('core') or {}).get('value'),d['roofline']['conv_launch_ms_per_step'])")"
  done
done
