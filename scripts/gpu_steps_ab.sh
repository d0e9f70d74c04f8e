set -o pipefail
mkdir -p gpurun_out
A="--no-cpu --stage-scans 8 --target-steps 0 --no-h2d --no-tile1 --multi= --multi-1m="
for i in 1 2; do
for K in 40 200; do
timeout -k 10 200 python bench.py $A --steps $K > gpurun_out/st_${K}_$i.json 2>/dev/null || exit 1
python -c "import json; d=json.load(open('gpurun_out/st_${K}_$i.json')); print('$K', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline_k_iekf'].get('P_k_source', d['roofline_k_iekf'].get('P_k_mean')))"
done
done
