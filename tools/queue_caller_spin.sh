set -u
cd "$GRAFT_REPO_ROOT"
for r in 1 2; do
for c in 0 3000 10000 40000; do
  echo "round=$r caller_spin_ns=$c"
  XRS_QUEUE_CALLER_SPIN_NS=$c timeout -k 10 60 tools/sync_bench 4096 queue 50 8 32 64 || exit 1
done; done
