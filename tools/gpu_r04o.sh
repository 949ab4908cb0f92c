set -e
for p in none matmul copy none; do timeout -k 10 120 python tools/step_times.py --preload $p; done
