set -o pipefail
O=gpurun_out/xdev; mkdir -p $O
for f in exact sampled; do
  timeout -k 10 300 python3 bench.py --op exchange --exchange-form $f --steps 10 --warmup 2 > $O/x16_$f.json 2> $O/x16_$f.err || exit 1
  timeout -k 10 300 python3 bench.py --op exchange --exchange-form $f --width 8 --steps 10 --warmup 2 > $O/x8_$f.json 2> $O/x8_$f.err || exit 1
done
