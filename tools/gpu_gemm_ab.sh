#!/bin/bash
# fp32 GEMM A/B at the cfg3 shapes (tools/gemm_ab.py), one process per variant, each time-limited.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-gemm_ab}
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?; echo "$name $rc $(date +%T)" >> "$OUT/status.txt"
  [ $rc -eq 0 ] || { echo "FATAL $name $rc"; tail -30 "$OUT/$name.out"; tail -30 "$OUT/$name.err"; exit $rc; }
  cat "$OUT/$name.out"
}
for v in ${VARIANTS:-default}; do
  case $v in
    default) run ab_default 300 python tools/gemm_ab.py ${AB_ARGS:-} ;;
    *) run ab_$v 300 env $(echo $v | tr '+' ' ') python tools/gemm_ab.py ${AB_ARGS:-} ;;
  esac
done
