# round-6 GPU job: q16 tier + 100M store pass (kernel trace), then the node-memory and config-4
# runs. A step that fails by exit status 1 (a test or check) is recorded and the job goes on; a
# time limit, abort or signal (status > 1) ends the job there.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
step() {  # name, command...
  local n=$1; shift
  echo "== $n start $(date +%T)"
  "$@"
  local rc=$?
  echo "== $n rc $rc $(date +%T)"
  if [ $rc -gt 1 ]; then exit $rc; fi
  return 0
}
step q16 bash tools/jobs/r6_q16b.sh
step mem bash tools/jobs/r6_mem.sh
