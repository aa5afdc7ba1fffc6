set -o pipefail; cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
T=${TAG:-r05zx}; export TMPDIR=/tmp
for R in 1 2; do for A in 0 512 4 64; do
  ME_HIP_LIB=libme_hip_tune.so ME_BW_ABL=$A timeout -k 10 100 python3 tools/ssd_ab.py --frames 16 --configs 1080p --tag abl$A --ms 300 >> gpurun_out/${T}_abl.jsonl 2>> gpurun_out/${T}_abl.err; rc=$?; echo "abl $A rc=$rc"; case $rc in 0|1) ;; *) exit $rc;; esac
done; done
python3 - <<'PY'
import json,collections
d=collections.defaultdict(list)
for l in open('gpurun_out/r05zx_abl.jsonl'):
    r=json.loads(l); d[r['tag']].append(round(r['us_per_frame'],2))
for k,v in sorted(d.items()): print(k, v)
PY
