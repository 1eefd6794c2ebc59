# Sourced by GPU scripts: `step <cmd...>` runs one GPU step; a plain failure (exit 1: a
# comparison or test failed) lets the script go on, anything else (time limit 124 / 137, abort
# 134, segfault 139, ...) ends the script there -- no further GPU work after a fault.
step() {
  echo "=== $* ($(date +%T))"
  "$@"
  local rc=$?
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP: rc=$rc at: $*"; exit $rc; fi
  [ $rc -eq 1 ] && echo "(step failed: rc=1)"
  return 0
}
