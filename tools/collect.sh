#!/usr/bin/env bash
# Copy a closing run's artifacts (tools/closing_run.sh -> gpurun_out/<round>_fin)
# into profiles/ under the round's prefix: per config the unprofiled line, the
# line printed under rocprofv3 and that run's kernel stats; the roofline
# checks, the PMC traffic table, the GPU suite log and the smoke log.
# usage: tools/collect.sh ROUND [INDIR]     (ROUND e.g. r05)
set -e
cd "$(dirname "$0")/.."
R=${1:?round prefix, e.g. r05}
I=${2:-gpurun_out/${R}_fin}
P=profiles
stats() { find "$1" -name '*kernel_stats.csv' | head -1; }
for d in "$I" "$I/nopmc"; do
  [ -d "$d" ] || continue
  for f in "$d"/*_noprof.json; do
    [ -f "$f" ] || continue
    n=$(basename "$f" _noprof.json)
    t=$n
    # a second line of a config (the unprofiled pass of a later call): keep the first
    # (the first line: this call's PMC'd lines or PART=1's)
    [ "$d" = "$I/nopmc" ] && { [ -f "$I/${n}_noprof.json" ] || [ -f "gpurun_out/${R}_fin/${n}_noprof.json" ]; } && t=${n}b
    cp "$f" "$P/${R}_${t}_noprof.json"
    [ -f "$d/$n.json" ] && cp "$d/$n.json" "$P/${R}_$t.json"
    s=$(stats "$d/trace_$n"); [ -n "$s" ] && cp "$s" "$P/${R}_${t}_kernel_stats.csv"
  done
done
# the roofline checks per part: the join lines, the op lines (PART=2), 1024M (PART=3)
case "$I" in *_fin2) rs=_ops ;; *_fin3) rs=_n1024 ;; *) rs= ;; esac
[ -f "$I/roofcheck.json" ] && cp "$I/roofcheck.json" "$P/${R}_roofcheck$rs.json"
[ -f "$I/nopmc/roofcheck.json" ] && cp "$I/nopmc/roofcheck.json" "$P/${R}_roofcheck_nopmc.json"
[ -f "$I/pmc_traffic.json" ] && cp "$I/pmc_traffic.json" "$P/pmc_traffic.json"
[ -f "$I/pytest_gpu.txt" ] && cp "$I/pytest_gpu.txt" "$P/${R}_pytest_gpu.txt"
[ -f "$I/smoke.txt" ] && cp "$I/smoke.txt" "$P/${R}_smoke.txt"
[ -f "$I/sq_join8.txt" ] && cp "$I/sq_join8.txt" "$P/${R}_sq_join8.txt"
ls -la "$P" | grep -c "${R}_"
