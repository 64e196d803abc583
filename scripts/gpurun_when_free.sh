# Submit one gpurun call, re-submitting only while gpurun answers 3 (no box or slot free: nothing ran, nothing
# charged), at most TRIES times, WAIT seconds apart.  Any other answer (the command ran, or was refused) ends it.
#   bash scripts/gpurun_when_free.sh LOG 'bash scripts/gpu_x.sh'
LOG=$1
CMD=$2
for i in $(seq 1 ${TRIES:-10}); do
  /usr/local/graft/bin/gpurun --timeout ${LIMIT:-1150} -- "$CMD" > "$LOG" 2>&1
  rc=$?
  [ $rc -ne 3 ] && { echo "rc=$rc after $i submissions"; exit $rc; }
  sleep ${WAIT:-180}
done
echo "no box after ${TRIES:-10} submissions"
exit 3
