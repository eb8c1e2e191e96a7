"""Seeded synthetic batches: the bench's workload generator (BASELINE.md "Inputs").

splitmix64 over a seed taken from the reference bench's XorShift seed bytes
(benchmarking/src/blake2f_circuit_bench.rs:41-44 starts 0x59, 0x62, 0xbe, 0x5d).
h, m, t uniform u64; f Bernoulli(1/2); rounds fixed or drawn from a mix.
"""
import numpy as np

from .layout import INPUT_DTYPE

DEFAULT_SEED = 0x5962be5d


def _mix(z):
    with np.errstate(over="ignore"):
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def _splitmix64(state, n):
    """n splitmix64 outputs starting from `state` (vectorised, wraps mod 2^64)."""
    with np.errstate(over="ignore"):
        idx = np.arange(1, n + 1, dtype=np.uint64)
        z = np.uint64(state) + idx * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def batch(n, rounds=12, seed=DEFAULT_SEED, first=0, rounds_mix=None):
    """Instances [first, first+n) of the seeded stream (so shards of one batch agree with
    the whole batch). rounds_mix: sequence of rounds values drawn uniformly per instance."""
    n = int(n)
    words_per = 8 + 16 + 2 + 2
    with np.errstate(over="ignore"):
        start = np.uint64(seed) + np.uint64(first * words_per) * np.uint64(0x9E3779B97F4A7C15)
    z = _splitmix64(start, n * words_per).reshape(n, words_per)
    out = np.zeros(n, dtype=INPUT_DTYPE)
    out["h"] = z[:, 0:8]
    out["m"] = z[:, 8:24]
    out["t"] = z[:, 24:26]
    out["f"] = (z[:, 26] >> np.uint64(63)).astype(np.uint32)
    if rounds_mix is None:
        out["rounds"] = rounds
    else:
        mix = np.asarray(rounds_mix, dtype=np.uint32)
        out["rounds"] = mix[(z[:, 27] % np.uint64(len(mix))).astype(np.int64)]
    return out


def rounds_of(n, rounds=12, seed=DEFAULT_SEED, rounds_mix=None):
    """The `rounds` field of instances [0, n) of the same stream, without generating the
    other words (shard planning of a large batch needs only the row map): an INPUT_DTYPE
    array whose other fields are zero."""
    n = int(n)
    out = np.zeros(n, dtype=INPUT_DTYPE)
    if rounds_mix is None:
        out["rounds"] = rounds
        return out
    words_per = 8 + 16 + 2 + 2
    with np.errstate(over="ignore"):
        k = (np.arange(n, dtype=np.uint64) + np.uint64(1)) * np.uint64(words_per)
        z = _mix(np.uint64(seed) + k * np.uint64(0x9E3779B97F4A7C15))
    mix = np.asarray(rounds_mix, dtype=np.uint32)
    out["rounds"] = mix[(z % np.uint64(len(mix))).astype(np.int64)]
    return out
