"""ORACLE / TEST INFRASTRUCTURE ONLY — never imported by the product path.

ctypes loader for oracle/torch_pow.c (the bit-level restatement of torch's CPU
`int64 counts ** (1/T)`, train_torch.py:192). The C file is compiled on first use with
gcc into oracle/_build/ (gcc is in the image here and on the GPU box)."""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "torch_pow.c")
OUT = os.path.join(HERE, "_build", "libtorchpow.so")
# torch's cpu_kernel_vec handles 2 x Vectorized<float>::size() elements per iteration; the reference
# fixtures were generated on an AVX512 host (16-float vectors -> 32)
VEC_BLOCK = 32
_lib = None


def build():
    if not os.path.exists(OUT) or os.path.getmtime(OUT) < os.path.getmtime(SRC):
        os.makedirs(os.path.dirname(OUT), exist_ok=True)
        tmp = OUT + f".{os.getpid()}.tmp"
        subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-shared", "-fPIC", "-o", tmp, SRC, "-lm"], check=True)
        os.replace(tmp, OUT)
    return OUT


def lib():
    global _lib
    if _lib is None:
        L = ctypes.CDLL(build())
        L.mz_torch_pow_counts.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_longlong, ctypes.c_double,
                                          ctypes.c_int, ctypes.c_longlong, ctypes.c_longlong, ctypes.c_longlong]
        L.mz_sleef_powf_u10.argtypes = [ctypes.c_float, ctypes.c_float]
        L.mz_sleef_powf_u10.restype = ctypes.c_float
        _lib = L
    return _lib


GRAIN_SIZE = 32768  # at::internal::GRAIN_SIZE: TensorIterator::for_each runs serially below it


def pow_chunk(n_total, threads, grain=GRAIN_SIZE):
    """Elements per intra-op thread chunk of torch's CPU pow over a tensor of n_total elements run with
    `threads` threads (TensorIterator::for_each -> at::parallel_for: serial below the grain size or on
    one thread, else min(threads, ceil(n / grain)) chunks of ceil(n / chunks) elements)."""
    if threads <= 1 or n_total < grain:
        return n_total
    num = min(threads, -(-n_total // grain))
    return -(-n_total // num)


def pow_counts(counts, e, vec_block=VEC_BLOCK, env_offset=0, n_envs_total=None, threads=1):
    """counts int64 (B, 3) ** e -> f32 (B, 3), for envs [env_offset, env_offset + B) of the reference's
    whole (n_envs_total, 3) batch tensor (default: counts is the whole tensor), evaluated by a torch
    process with `threads` intra-op threads (matters from 32768 elements on)."""
    c = np.ascontiguousarray(counts, dtype=np.int64)
    out = np.empty(c.shape, dtype=np.float32)
    nt = 3 * (c.shape[0] + env_offset if n_envs_total is None else n_envs_total)
    lib().mz_torch_pow_counts(c.ctypes.data, out.ctypes.data, c.size, float(e), int(vec_block), 3 * env_offset, nt,
                              pow_chunk(nt, threads))
    return out
