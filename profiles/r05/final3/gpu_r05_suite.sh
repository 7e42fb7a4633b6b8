#!/bin/bash
# Round-5 closing check: the whole -m gpu suite and smoke on the round's last tree.
OUT=gpurun_out/${1:-r05_suite}
mkdir -p $OUT
export TMPDIR=/tmp
step() {
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name $rc" >> $OUT/status
  if [ $rc -gt 1 ]; then echo "stopping after $name ($rc)" >> $OUT/status; exit 0; fi
}
step suite 1100 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
echo done >> $OUT/status
