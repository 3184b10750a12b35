set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r6z2; mkdir -p $O
RR="python3 -m analyzer_amd.runtime.rerate --matches 1e9 --players 1e7 --window 1.6e7"
for r in 1 2; do
  rm -rf /tmp/cka; timeout -k 10 300 $RR --checkpoint-dir /tmp/cka --checkpoint-every 8 > $O/ck8_$r.log 2>&1 || exit 1
  timeout -k 10 300 $RR > $O/nock_$r.log 2>&1 || exit 1
  timeout -k 10 300 $RR --records none > $O/norec_$r.log 2>&1 || exit 1
done
df -h /tmp | tail -1
for f in $O/*.log; do n=$(basename $f .log); echo "$n $(tail -1 $f | grep -o '"seconds": [0-9.]*')"; done | sort
