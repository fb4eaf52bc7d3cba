"""Throughput of the batched Atari frame pipeline (acmi_atari_stack): N envs' last two
raw 210x160x3 frames -> max, gray, INTER_AREA 84x84, 4-frame stack update.
Algorithmic HBM bytes per env-step: 2 raw frames (201,600) + stack read and write
(2 x 28,224) = 258,048."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'actor-critic_amd'))

from actorcritic.envs.atari import wrappers

BYTES_PER_ENV = 2 * 210 * 160 * 3 + 2 * 84 * 84 * 4


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--envs', type=int, default=512)
    ap.add_argument('--iters', type=int, default=200)
    a = ap.parse_args()
    pipe = wrappers.AtariFramePipeline(a.envs)
    pipe.raw.random_(0, 256)
    term = (torch.rand(a.envs, device=pipe.device) < 0.01).to(torch.uint8)
    pipe.reset()
    for _ in range(10):
        pipe.step(term)
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record(s)
    for _ in range(a.iters):
        pipe.step(term)
    e1.record(s)
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / a.iters
    gbs = a.envs * BYTES_PER_ENV / (us * 1e-6) / 1e9
    print(json.dumps({'envs': a.envs, 'us_per_step': us, 'env_steps_per_s': a.envs / (us * 1e-6),
                      'algorithmic_GBps': gbs, 'frac_of_8TBps': gbs / 8000}))


if __name__ == '__main__':
    main()
