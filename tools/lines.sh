#!/usr/bin/env bash
# Roofline artifacts: per config, in ONE command on one box,
#   NAME_noprof.json   the bench line without the profiler (CPU baseline on)
#   NAME.json          the line printed by rocprofv3 --kernel-trace --stats
#   trace_NAME/        that run's kernel stats / trace CSV
#   fetch_/write_NAME  FETCH_SIZE and WRITE_SIZE passes -> pmc_traffic.json
# then tools/roofcheck.py compares each line's frac with the rocprof average.
# usage: tools/lines.sh OUTDIR NAME:args [NAME:args ...]
# The first failure ends the script (no GPU step after a failed one).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=$1; shift
mkdir -p "$OUT"
[ -f profiles/pmc_traffic.json ] && cp profiles/pmc_traffic.json "$OUT/pmc_traffic.json"
NAMES=()
for cfg in "$@"; do
  name=${cfg%%:*}; args=${cfg#*:}; NAMES+=("$name")
  key=$(python3 - "$args" <<'EOF'
import sys
a = sys.argv[1].split()
def get(f, d):
    return a[a.index(f) + 1] if f in a else d
op = get("--op", "join")
if op == "join":
    n = get("--n", "128000000"); w = get("--width", "16"); dist = get("--dist", "uniform")
    pay = get("--payload", "rowid")
    print(f"n{n}_w{w}_{dist}" + ("" if pay == "rowid" else f"_{pay}"))
else:
    w = get("--width", "8")
    n = int(get("--n", str(65536 if op == "merge" else 1 << 27)))
    if op == "merge":
        n *= int(get("--fanin", "64"))
    print(f"{op}_n{n}_w{w}")
EOF
)
  timeout -k 10 300 python3 bench.py $args ${CPU_ARGS:-} > "$OUT/${name}_noprof.json" 2> "$OUT/${name}_noprof.err" \
    || { echo "FAIL noprof $name"; tail -5 "$OUT/${name}_noprof.err"; exit 1; }
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_$name" -o run -- python3 bench.py $args --no-cpu-baseline > "$OUT/$name.json" 2> "$OUT/$name.err" \
    || { echo "FAIL trace $name"; tail -5 "$OUT/$name.err"; exit 1; }
  if [ -z "${NO_PMC:-}" ]; then
    timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/fetch_$name" -o run -- python3 bench.py $args --no-cpu-baseline > "$OUT/fetch_$name.log" 2>&1 \
      || { echo "FAIL fetch $name"; exit 1; }
    timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/write_$name" -o run -- python3 bench.py $args --no-cpu-baseline > "$OUT/write_$name.log" 2>&1 \
      || { echo "FAIL write $name"; exit 1; }
    python3 tools/make_traffic.py "$key" "$OUT/fetch_$name" "$OUT/write_$name" "$OUT/pmc_traffic.json" > /dev/null || exit 1
  fi
  echo "$name [$key] $(head -c 150 "$OUT/${name}_noprof.json")"
done
python3 tools/roofcheck.py "$OUT" "${NAMES[@]}" > "$OUT/roofcheck.json" && cat "$OUT/roofcheck.json"
