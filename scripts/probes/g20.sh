set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/${TAG:-r5z}
mkdir -p $out
for v in "MOOSEX_WSUM_FUSED=0" "MOOSEX_DEFER_DOT_TRUNC=0" "MOOSEX_MERGE_ROUNDS=0" "MOOSEX_X=1"; do
  env $v timeout -k 10 120 python scripts/probes/lr_parties_prof.py --runs 3 > $out/$v.json 2> $out/$v.err
  echo "$v rc=$?" >> $out/summary.txt
done
