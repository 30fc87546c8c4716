set -u
mkdir -p gpurun_out
for nb in 256 192 128 64; do
XA_AC_BLOCKS=$nb timeout -k 10 120 python bench.py --steps 30 --warmup 5 --cpu-baseline-seconds 0 > gpurun_out/b_nb$nb.log 2>&1 || exit 1
python -c "
import json; d=json.loads(open('gpurun_out/b_nb$nb.log').read().strip().splitlines()[-1]); print($nb, d['ms_per_step'], d['update_ms'], d['roofline']['launch_ms'])"
done
