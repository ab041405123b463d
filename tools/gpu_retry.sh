# Retry a gpurun call only while it reports "no box / transient" (exit 3); any other result
# ends it. Usage: bash tools/gpu_retry.sh '<command>' <log> [attempts] [limit_s]
cmd="$1"; log="$2"; n="${3:-40}"; lim="${4:-1200}"
for i in $(seq 1 "$n"); do
  timeout $((lim + 1500)) /usr/local/graft/bin/gpurun --timeout "$lim" -- "$cmd" > "$log" 2>&1
  rc=$?
  echo "attempt $i rc=$rc $(date +%H:%M:%S)" >> "$log.attempts"
  [ $rc -ne 3 ] && break
  sleep 120
done
echo "final rc=$rc" >> "$log.attempts"
