cd "${GRAFT_REPO_ROOT}"
for i in 1 2; do for v in 512 256; do
ACMI_AF_SLOTS=$v timeout -k 10 120 python bench.py --forward bf16 --num-actions 18 --envs-per-gpu 1024 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/c4.json 2>gpurun_out/c4.err || exit $?
python -c "
import json; d=json.loads(open('gpurun_out/c4.json').read().strip().splitlines()[-1]); print('$v', round(d['value']), round(d['update_ms'],3))"
done; done
