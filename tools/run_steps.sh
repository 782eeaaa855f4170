#!/bin/bash
# Run GPU steps in order (each "name|command", each under its own timeout inside the command);
# a step that times out, aborts or faults (124, 134, 137, 139) ends the batch, other failures
# are reported and the batch goes on. Usage: tools/run_steps.sh "name|cmd" ...
for s in "$@"; do
  name=${s%%|*}; cmd=${s#*|}
  echo "== $name"
  bash -c "$cmd"
  rc=$?
  echo "== $name rc=$rc"
  case $rc in 124|134|137|139) echo "stopping after $name"; exit $rc;; esac
done
