"""CPU: the integrate kernels' tiling/binning logic (csrc/dm_ray.h, run by a
sequential host emulation of the four kernels, tests/native/emulate.cpp)
reproduces the oracle bit for bit.  Pins the kernel geometry without a GPU."""
import ctypes
import math
import os
import subprocess

import numpy as np
import pytest

import cases
from golden_io import load_case

HERE = os.path.dirname(os.path.abspath(__file__))
NATIVE = os.path.join(HERE, "native")


@pytest.fixture(scope="module")
def emu():
    subprocess.run(["make", "-s", "-C", NATIVE], check=True)
    lib = ctypes.CDLL(os.path.join(NATIVE, "libemu.so"))
    f = lib.emu_integrate
    i32, d, fl, vp = ctypes.c_int32, ctypes.c_double, ctypes.c_float, ctypes.c_void_p
    f.argtypes = [i32, i32, i32, d, d, d] + [fl] * 8 + [vp, vp, i32, vp, i32, vp, vp, vp, vp, vp, i32]
    return lib


class EmuMap:
    def __init__(self, lib, p, chunk_len=0):
        self.lib, self.p, self.chunk_len = lib, p, chunk_len
        R = int(p.band_rows) if p.band_rows > 0 else int(p.height - p.band_row0)
        self.L = np.zeros((R, int(p.width)), np.float32)
        self.state = np.full((R, int(p.width)), -1, np.int8)

    def integrate(self, poses, ranges, amin, inc):
        p = self.p
        poses = np.asarray(poses, np.float64).reshape(-1, 3)
        ranges = np.ascontiguousarray(ranges, np.float32).reshape(poses.shape[0], -1)
        S, N = ranges.shape
        pose4 = np.array([[x, y, math.cos(t), math.sin(t)] for x, y, t in poses], np.float64).reshape(S, 4)
        amin32, inc32 = float(np.float32(amin)), float(np.float32(inc))
        trig = np.array([[math.cos(amin32 + i * inc32), math.sin(amin32 + i * inc32)]
                         for i in range(N)], np.float64).reshape(N, 2)
        U, T, G = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
        ptr = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
        rc = self.lib.emu_integrate(int(p.width), self.L.shape[0], int(p.band_row0), p.origin_x, p.origin_y,
                               p.resolution, p.range_min, p.range_max, p.l_occ, p.l_free, p.l_min,
                               p.l_max, p.occ_thresh, p.free_thresh, ptr(self.L), ptr(self.state), S,
                               ptr(pose4), N, ptr(ranges), ptr(trig), ctypes.byref(U),
                               ctypes.byref(T), ctypes.byref(G), self.chunk_len)
        assert rc == 0, f"emulation check {rc} failed (-10x: piece walk vs closed form)"
        return int(U.value), int(T.value)


@pytest.mark.parametrize("name", ["tiny64", "c1_room", "ragged", "offgrid"])
def test_emulated_kernels_match_golden(emu, name):
    d = np.load(os.path.join(HERE, "golden", "oracle_golden.npz"))
    c = load_case(d, name)
    m = EmuMap(emu, c["params"], 0)
    for k, (poses, ranges) in enumerate(c["batches"]):
        assert m.integrate(poses, ranges, c["amin"], c["inc"]) == tuple(c["counts"][k])
    np.testing.assert_array_equal(m.L.view(np.uint32), c["L"].view(np.uint32))
    np.testing.assert_array_equal(m.state, c["state"])


@pytest.mark.parametrize("W,H,S,N,res,seed,r0,rows", [
    (257, 513, 6, 700, 0.05, 4, 0, 0), (1000, 300, 4, 2048, 0.02, 5, 0, 0),
    (96, 96, 12, 256, 0.1, 6, 0, 0), (300, 700, 8, 600, 0.05, 7, 320, 192),
    (500, 500, 3, 3000, 0.01, 8, 128, 0)])
@pytest.mark.parametrize("chunk_len", [0, 64, 97])
def test_emulated_kernels_random(emu, oracle_lib, W, H, S, N, res, seed, r0, rows, chunk_len):
    """chunk_len > 0: beams enumerated in k-ranges as k_beam_prep / k_scatter
    do for small batches (dm_integrate_chunks)."""
    p = cases.make_params(W, H, resolution=res, band_row0=r0, band_rows=rows)
    om = oracle_lib.OracleMap(p)
    m = EmuMap(emu, p, chunk_len)
    for k in range(2):
        poses, ranges, amin, inc = cases.random_scans(seed * 10 + k, p, S, N,
                                                      spread=4.0 if seed == 6 else 1.0)
        assert m.integrate(poses, ranges, amin, inc) == om.integrate(poses, ranges, amin, inc)
    np.testing.assert_array_equal(m.L.view(np.uint32), om.L.view(np.uint32))
    np.testing.assert_array_equal(m.state, om.state)
