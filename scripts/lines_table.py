"""BASELINE.md §3 table rows from a config_lines.sh output directory:
   python scripts/lines_table.py gpurun_out/r04_lines"""
import glob
import json
import os
import sys

NAMES = [
    ('configs1_a2c_32x5', 'Breakout A2C, 32 envs × 5 steps, 1 GPU (configs[1])'),
    ('configs2_acktr_32x20', 'Breakout ACKTR, 32 envs × 20 steps, invert every 10, 1 GPU (configs[2])'),
    ('configs3_shard_acktr_512x20', 'Breakout ACKTR, 512 envs × 20 per GPU (configs[3] shard, the bench default)'),
    ('configs4_shard_bf16_1024x20_a18', 'Atari ACKTR shard, 1024 envs × 20, A = 18, bf16 fwd / fp32 factors, one game (configs[4] shard)'),
    ('configs4_mixed_atari57_1024x20_a18_bf16', 'Mixed Atari-57 ACKTR shard, 1024 envs × 20, A = 18, bf16 fwd / fp32 factors (configs[4] shard, `--games atari57`)'),
]


def main(d):
    for key, label in NAMES:
        f = os.path.join(d, key + '.json')
        if not os.path.exists(f):
            print('| {} | missing |'.format(label))
            continue
        x = json.loads(open(f).read().strip().splitlines()[-1])
        cb = x.get('cpu_baseline') or {}
        cpu = cb.get('value')
        print('| {} | {:,.0f} | {:.1f} | {:,.0f} | {:.2f} | {:,.0f}× | {:.2f} |'.format(
            label, cpu or 0, cb.get('update_ms', 0), x['value'], x.get('update_ms', 0),
            (x['value'] / cpu) if cpu else 0, x['roofline']['frac']))


if __name__ == '__main__':
    main(sys.argv[1])
