#!/bin/bash
# One GPU session as a list of named steps, each under its own time limit -- the one script every GPU call of
# round 6 runs (the per-session scripts of rounds 2-5 are gone; their outputs stay under profiles/rNN/):
#
#   tools/gpu_steps.sh OUTDIR 'name|seconds|command' ['name|seconds|command' ...]
#
# Each step's stdout and stderr go to OUTDIR/name.log, its exit code to OUTDIR/status.  Exit code 1 (a failing
# test, a bench that refuses an unverified result) lets the session go on; anything above 1 -- a fault, an
# abort, a time limit (124/137) -- ends it there, so nothing more touches the GPU after trouble.
OUT=$1
shift
mkdir -p "$OUT"
export TMPDIR=/tmp
for spec in "$@"; do
  name=${spec%%|*}
  rest=${spec#*|}
  secs=${rest%%|*}
  cmd=${rest#*|}
  echo "$name start $(date +%T)" >> "$OUT/status"
  timeout -k 10 "$secs" bash -c "$cmd" > "$OUT/$name.log" 2>&1
  rc=$?
  echo "$name $rc $(date +%T)" >> "$OUT/status"
  if [ $rc -gt 1 ]; then
    echo "stopping after $name ($rc)" >> "$OUT/status"
    exit 0
  fi
done
echo done >> "$OUT/status"
