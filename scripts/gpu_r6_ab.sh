# Same-box A/B of bench variants: each argument is "tag|ENV=VAL ENV=VAL" (tag alone: the default),
# two alternating rounds; prints img/s, ms/step, conv launch ms and the G / D / VGG19 conv ms.
set -o pipefail
O=gpurun_out/r6_ab_${TAG:-x}
mkdir -p $O
export TMPDIR=/tmp
L=$PWD/denoise-gan_amd/lib
B="python bench.py --steps 30 --warmup 8 --no-cpu-baseline --no-twin --no-core --no-pmc-leg $EXTRA"
for r in 1 2; do
  for v in "$@"; do
    tag=${v%%|*}; envs=""; [ "$v" != "$tag" ] && envs=${v#*|}
    envs=${envs//@L/$L}
    env $envs timeout -k 10 300 $B > $O/${tag}_$r.json 2> $O/${tag}_$r.err || exit 1
    echo "$tag $r $(python -c "
import json;d=json.loads(open('$O/${tag}_$r.json').read().strip().splitlines()[-1]);r=d['roofline'];n=r['by_net']
print(d['value'],d['ms_per_step'],r['conv_launch_ms_per_step'],'G',n['G']['ms_per_step'],'D',n['D']['ms_per_step'],'V',n.get('vgg19',{}).get('ms_per_step'),'p2p',r['p2p_convs']['frac'])")"
  done
done
