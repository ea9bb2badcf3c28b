set -e
cd $GRAFT_REPO_ROOT
for v in v1 v2 v3 v4; do
  for z in 0 1.1; do
    echo "== $v zipf $z"
    timeout -k 10 120 tools/tune_c5u_$v 125000000 8 24 $z
  done
done
