"""Diagnostic: per-phase cycle shares of the rollout and update kernels (libpgm_stamps.so).
Usage (GPU box): PGM_LIB=pgmorl_amd/libpgm_stamps.so python scripts/stamps.py"""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from pgmorl_amd import _lib
from pgmorl_amd.policy import new_policy
from pgmorl_amd.runtime import TaskBatch

ENV = os.environ.get('ENV', 'MO-Walker2d-v2')
HUM = 'Humanoid' in ENV
P, N, T = int(os.environ.get('P', 20 if HUM else 40)), 8 if HUM else 4, int(os.environ.get('T', 2048))
tb = TaskBatch(ENV, P, num_processes=N, num_steps=T)
for p in range(P):
    tb.set_task(p, new_policy(tb.O, tb.A, tb.K).state_dict(), {}, None, [0.5, 0.5])
tb.env_reset()
L = _lib.lib()
buf = (C.c_ulonglong * 64)()  # per-phase accumulators (ids < 24)
SB = int(os.environ.get('STAMP_BLOCK', 0))  # workgroup sampled (update SPLIT: 2p = critic, 2p+1 = actor)
UNITS = ('rollout', 'update', 'mfma', 'lanes', 'wide', 'wupd', 'fs')
for name in UNITS:
    getattr(L, f'pgm_debug_stamps_{name}')(buf, 1)
    getattr(L, f'pgm_debug_stamp_block_{name}')(SB)
tb.iteration(0, 3e-4)
torch.cuda.synchronize()
names = {0: "loop/top", 1: 'policy fwd', 2: 'store val + sample', 3: 'logp + dynamics', 4: 'vecnorm stats',
         5: 'vecnorm emit', 10: 'policy L2 (in fwd)'}
mnames = {0: 'stage rows', 1: 'pass end sync', 2: 'grad image rounds', 3: 'Adam', 8: 'sumsq', 9: 'norm exchange',
          10: 'half image publish + drain', 11: 'flag hand-off + image gather',
          4: 'tile: L1 + L2 fwd', 5: 'tile: heads + loss', 6: 'tile: gWh, dH2, gW2', 7: 'tile: dH1, gW1',
          12: 'image: lane sums', 13: 'image: stage 0 work', 14: 'image: stage 1 work', 15: 'image: stage 0 barrier',
          16: 'tile: heads (VALU)', 17: 'tile: loss + dO tile', 18: 'tile: dO fence', 5: 'tile: head column sums', 19: 'Adam math (MODE 2)'}
lnames = {0: 'loop/top', 1: 'actor fwd', 6: 'sample', 7: 'dynamics', 2: 'accumulators + row', 3: 'barrier',
          4: 'stats', 5: 'emit'}
wnames = {0: 'noise + layer-1 slices', 1: 'barrier A', 2: 'L1 sum, L2, head, draw', 3: 'barrier C',
          4: 'dynamics', 5: 'objective wave sums', 6: 'reset + ob_rms + emit', 7: 'stats wave + barrier D'}
unames = {0: 'layer 1 (L2 stream)', 1: 'layer 2 + tanh', 2: 'heads + loss', 3: 'gWh, dH2, gW2, dH1',
          4: 'pass barrier 1', 5: 'dW1 contraction', 6: 'pass barrier 2', 7: 'small-image reduction',
          8: 'publish + flag wait', 9: 'gather partner', 10: 'sumsq + norm hand-off',
          12: 'Adam: layer-1 slice (HBM)', 13: 'Adam: slice publish + image (LDS)', 14: 'Adam: slice drain',
          15: 'Adam: slice flag wait', 11: 'Adam: partner slices -> copy'}
fnames = {0: 'put W1/vec + L1', 11: 'put W2/Wh', 12: 'B1 wait', 1: 'L2 + H2 write', 13: 'B2 wait',
          14: 'Wh reads + head MFMAs', 15: 'loss VALU', 2: 'group sums', 3: 'B2b + gWh, dH2, gW2',
          4: 'B3 + dH1, gW1', 5: 'publish + drain + barrier', 6: 'image flag poll (+ row DMA)',
          7: 'reduce-scatter loads + sumsq', 8: 'norm granules', 9: 'Adam + publish + param poll', 10: 'gather issue'}
for name, steps in (('rollout', T), ('update', 320), ('mfma', 320), ('lanes', T), ('wide', T), ('wupd', 320), ('fs', 320)):
    if name == 'fs':
        names = fnames
    if name == 'wupd':
        names = unames
    if name == 'mfma':
        names = mnames
    if name == 'lanes':
        names = lnames
    if name == 'wide':
        names = wnames
    getattr(L, f'pgm_debug_stamps_{name}')(buf, 1)
    v = np.array(list(buf), dtype=np.float64)
    tot = v.sum()
    if tot == 0:
        continue
    print(f'== {name}: total {tot:.3e} cycles over {steps} iterations ({tot / steps:.0f} cycles/iter)')
    for i in np.nonzero(v)[0]:
        print(f'  phase {i:2d} {names.get(i, ""):22s} {v[i] / steps:10.0f} cycles/iter  {100 * v[i] / tot:5.1f}%')
