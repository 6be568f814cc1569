# A/B of library builds (gpurun, repo root): one timing script alternated over the builds given as
# arguments (HALO_LIB), two interleaved runs each, so box-to-box drift hits every build alike.
#   bash tools/ab.sh msm  <lib> ...    headline bench (MSM + NTT legs, no CPU leg): ms/step, k_acc
#   bash tools/ab.sh msm24 <lib> ...   the same plus the 2^24 sizes leg (pipelined MSMs, NTT pair)
#   SIZES="22 23 24" bash tools/ab.sh ntt  <lib> ...    NTT pairs (tools/ntt_time.py)
#   SIZES="2 6 10"   bash tools/ab.sh pcdl <lib> ...    pcdl::open sweep (tools/pcdl_open_time.py)
#   SIZES="16 20"    bash tools/ab.sh ipa  <lib> ...    IPA openings (tools/ipa_time.py)
#   SIZES="16"       bash tools/ab.sh prove <lib> ...   naive_prover rounds (tools/prove_time.py, warm repetition)
set -o pipefail
cd $GRAFT_REPO_ROOT
what=$1; shift
O=gpurun_out/ab_$what; rm -rf $O; mkdir -p $O
for i in 1 2; do
  for lib in "$@"; do
    tag=$(basename $lib .so)_$i
    echo "== $tag"
    case $what in
      msm)
        HALO_LIB=$PWD/$lib timeout -k 10 200 python bench.py --no-cpu --sizes "" --ipa 0 --prove 0 --varbase 0 \
          --commit-batch 0 --pcdl "" --steps 20 > $O/$tag.json 2> $O/$tag.err || { tail -20 $O/$tag.err; exit 1; }
        python3 -c "
import json; d = json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); e = d['extra']
print('ms/step %.4f  k_acc %.3f  latency %.3f  ntt pair %.3f' % (d['ms_per_step'], d['roofline']['avg_launch_ms'],
      e['msm_single_latency_ms'], e['ntt']['pair_ms']))" ;;
      msm24)  # headline and the 2^24 sizes leg (8 pipelined after 4 warm-up)
        HALO_LIB=$PWD/$lib timeout -k 10 300 python bench.py --no-cpu --sizes 24 --ipa 0 --prove 0 --varbase 0 \
          --commit-batch 0 --batch-ntt 0 --pcdl "" --steps 20 > $O/$tag.json 2> $O/$tag.err || { tail -20 $O/$tag.err; exit 1; }
        python3 -c "
import json; d = json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); s = d['extra']['sizes']
print('ms/step %.4f  k_acc %.3f (alone %.3f) | 2^24 ms/msm %.2f  k_acc %.2f  single %.2f | ntt24 pair %.3f' % (d['ms_per_step'],
      d['roofline']['avg_launch_ms'], d['roofline']['isolated_launch_ms'], s['msm_2^24']['ms_per_msm'], s['msm_2^24']['k_acc_ms'],
      s['msm_2^24']['single_latency_ms'], s['ntt_2^24']['pair_ms']))" ;;
      ntt)
        HALO_LIB=$PWD/$lib timeout -k 10 200 python tools/ntt_time.py ${SIZES:-22 23 24} 2>&1 | tail -${NL:-3} || exit 1 ;;
      pcdl)
        HALO_LIB=$PWD/$lib timeout -k 10 200 python tools/pcdl_open_time.py ${SIZES:-2 4 6 8 10 12} 2>&1 | grep "^2^" \
          | sed 's/begin+eval.*rounds=/rounds=/' || exit 1 ;;
      ipa)
        HALO_LIB=$PWD/$lib REPS=2 timeout -k 10 300 python tools/ipa_time.py ${SIZES:-16 20} 2>&1 | grep "^open" || exit 1 ;;
      prove)
        HALO_LIB=$PWD/$lib timeout -k 10 200 python tools/prove_time.py ${SIZES:-16} 2>&1 | grep '"rep": 1' || exit 1 ;;
      *) echo "unknown: $what (msm | msm24 | ntt | pcdl | ipa | prove)"; exit 2 ;;
    esac
  done
done
