#!/usr/bin/env bash
# Copy the closing run's artifacts (tools/r04_final_c.sh -> gpurun_out/r04_fin)
# into profiles/ under the round-4 names: per config the unprofiled line, the
# line printed under rocprofv3 and that run's kernel stats; the roofline
# checks, the PMC traffic table, the GPU suite log and the smoke log.
set -e
cd "$(dirname "$0")/.."
I=${1:-gpurun_out/r04_fin}
P=profiles
stats() { find "$1" -name '*kernel_stats.csv' | head -1; }
for d in "$I" "$I/nopmc"; do
  [ -d "$d" ] || continue
  for f in "$d"/*_noprof.json; do
    [ -f "$f" ] || continue
    n=$(basename "$f" _noprof.json)
    t=$n
    # a second line of a config (the headline again, without PMC passes)
    [ "$d" = "$I/nopmc" ] && { [ -f "$I/${n}_noprof.json" ] || [ "$n" = join16 ]; } && t=${n}b
    cp "$f" "$P/r04_${t}_noprof.json"
    [ -f "$d/$n.json" ] && cp "$d/$n.json" "$P/r04_$t.json"
    s=$(stats "$d/trace_$n"); [ -n "$s" ] && cp "$s" "$P/r04_${t}_kernel_stats.csv"
  done
done
[ -f "$I/roofcheck.json" ] && cp "$I/roofcheck.json" "$P/r04_roofcheck${TAG:-}.json"
[ -f "$I/nopmc/roofcheck.json" ] && cp "$I/nopmc/roofcheck.json" "$P/r04_roofcheck_nopmc.json"
cp "$I/pmc_traffic.json" "$P/pmc_traffic.json"
[ -f "$I/pytest_gpu.txt" ] && cp "$I/pytest_gpu.txt" "$P/r04_pytest_gpu.txt"
[ -f "$I/smoke.txt" ] && cp "$I/smoke.txt" "$P/r04_smoke.txt"
tr=$(find "$I/trace_join16" -name '*kernel_trace.csv' | head -1)
[ -n "$tr" ] && python3 tools/timeline.py "$tr" 10 "$P/r04_join16_step_timeline.csv" k_join_begin || true
ls -la "$P" | grep r04_ | wc -l
