# A/B of MSM pipeline variants on the GPU box (run through gpurun from the repo root).
# usage: bash tools/ab_msm.sh "<ENV1>" "<ENV2>" ...   each ENV is a space-separated VAR=VAL list
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
for cfg in "$@"; do
  tag=$(echo "$cfg" | tr ' =/.' '_-__')
  env $cfg timeout -k 10 200 python bench.py --no-cpu --sizes "${AB_SIZES:-}" --ipa ${AB_IPA:-0} --prove ${AB_PROVE:-0} --steps 20 > gpurun_out/ab/$tag.json 2> gpurun_out/ab/$tag.err || { echo "FAIL $cfg"; tail -5 gpurun_out/ab/$tag.err; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open('gpurun_out/ab/$tag.json').read().strip().splitlines()[-1])
e=d['extra']; print('$cfg', 'ms/step %.3f'%d['ms_per_step'], 'acc %.3f'%d['roofline']['avg_launch_ms'], 'lat %.3f'%e['msm_single_latency_ms'], 'sync_ok', e['pipelined_equals_sync'], 'ntt %.3f'%e['ntt']['pair_ms'], 'ipa', (e.get('ipa_open') or {}).get('open_ms'))
"
done
