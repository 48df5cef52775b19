"""DIAGNOSTIC: walk rounds of k_tile_accum's items for C3 / C5 batches
(tools/native/piece_stats.cpp).  Usage: python tools/piece_stats.py [C3|C5:N]"""
import ctypes
import math
import os
import subprocess
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "distributed-autonomous-exploration-and-mapping_amd"))
from dm import synth  # noqa: E402

nat = os.path.join(REPO, "tools", "native")
so = os.path.join(nat, "libpiece_stats.so")
subprocess.run(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-ffp-contract=off", "-o", so,
                os.path.join(nat, "piece_stats.cpp")], check=True)
lib = ctypes.CDLL(so)
cfg = sys.argv[1] if len(sys.argv) > 1 else "C3"
if cfg == "C3":
    G, res, S, N = 16384, 0.05, 64, 4096
    half = G * res / 2
    world = synth.make_world(0, -half, -half, half, half)
    stream = synth.ScanStream(world, S, N, 500, region=(-half + 1, -half + 1, half - 1, half - 1))
    W = H = G
    ox = oy = -half
    rmax = 12.0
else:
    N = int(cfg.split(":")[1])
    world, W, H, res, ox, oy = synth.config_world("C5", 0)
    S = 64
    stream = synth.ScanStream(world, S, N, 7 + N)
    rmax = 12.0
inc = float(synth.ld06_angle_increment(N))
amin = float(synth.LD06_ANGLE_MIN)
amin32, inc32 = float(np.float32(amin)), float(np.float32(inc))
trig = np.array([[math.cos(amin32 + i * inc32), math.sin(amin32 + i * inc32)] for i in range(N)], np.float64)
tot = np.zeros(21)
for _ in range(3):
    poses, ranges = stream.next_batch()
    p4 = np.ascontiguousarray(synth.pose4(poses)[:, :4], np.float64)
    ranges = np.ascontiguousarray(ranges, np.float32)
    out = np.zeros(21)
    ptr = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    lib.piece_stats.argtypes = [ctypes.c_int32, ctypes.c_int32] + [ctypes.c_double] * 3 + [ctypes.c_float] * 2 + \
        [ctypes.c_int32, ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    lib.piece_stats(W, H, ox, oy, res, 0.02, rmax, S, ptr(p4), N, ptr(ranges), ptr(trig), ptr(out))
    tot += out
tot /= 3
names = ["plain", "flat", "sorted", "ideal", "pieces", "chunks", "waves", "tiles", "cells",
         "light_plain", "light_flat", "light_sorted", "light_chunks", "light_pieces"]
for n, v in zip(names, tot):
    print(f"{n:14s} {v:14.0f}")
print(f"critical path per chunk: plain {tot[16] / tot[5]:.1f} split {tot[17] / tot[5]:.1f} "
      f"wgflat {tot[18] / tot[5]:.1f} waterfill {tot[14] / tot[5]:.1f}; wave-steps: plain {tot[0]:.0f} split {tot[19]:.0f} wgflat {tot[20]:.0f} waterfill {tot[15]:.0f}")
print(f"mean len {tot[8] / tot[4]:.1f}; rounds per wave: plain {tot[0] / tot[6]:.1f} flat {tot[1] / tot[6]:.1f} "
      f"sorted {tot[2] / tot[6]:.1f} ideal {tot[3] / tot[6]:.1f}; pieces per chunk {tot[4] / tot[5]:.0f}, "
      f"waves per chunk {tot[6] / tot[5]:.2f}")
