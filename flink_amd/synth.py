"""Synthetic event streams of SURVEY.md §8(d), generated where they are consumed (torch, any device).

Counter-based: record i of a stream is a pure function of (seed, i) through splitmix64, so the GPU
engine, the CPU oracle and a Java SourceFunction can all produce identical streams.
  key   = splitmix64(seed_key ^ i) & (n_keys - 1)           (n_keys a power of two), or % n_keys
          Zipf(s): inverse CDF of ranks 1..n_keys at u = (splitmix64(seed_key ^ i) >> 11) / 2^53
  ts    = t0 + (i * 1000) // rate                            (rate = events per event-time second)
          out of order by D: minus splitmix64(3 ^ i) % (D + 1)
  value = (int64) splitmix64(seed_val ^ i)                   full range: the long sums wrap
          doubles: (splitmix64(seed_val ^ i) >> 11) / 2^53   in [0, 1)
"""
import torch

_GOLD = -7046029254386353131          # 0x9E3779B97F4A7C15 as int64
_C1 = -4658895280553007687            # 0xBF58476D1CE4E5B9
_C2 = -7723592293110705685            # 0x94D049BB133111EB


def _lsr(x, s):
    """logical right shift on int64 tensors"""
    return (x >> s) & ((1 << (64 - s)) - 1)


def splitmix64(x):
    z = x + _GOLD
    z = (z ^ _lsr(z, 30)) * _C1
    z = (z ^ _lsr(z, 27)) * _C2
    return z ^ _lsr(z, 31)


_zipf_cdf = {}


def zipf_cdf(n_keys, s, device):
    k = (n_keys, s, str(device))
    if k not in _zipf_cdf:
        ranks = torch.arange(1, n_keys + 1, dtype=torch.float64)
        cdf = torch.cumsum(ranks ** -s, 0)
        _zipf_cdf[k] = (cdf / cdf[-1]).to(device)
    return _zipf_cdf[k]


def stream(start, n, n_keys, rate, t0=0, seed_key=1, seed_val=2, device="cpu", value_type="i64", zipf=None, ooo=0):
    i = torch.arange(start, start + n, dtype=torch.int64, device=device)
    hk = splitmix64(i ^ seed_key)
    if zipf is not None:
        u = _lsr(hk, 11).to(torch.float64) / float(1 << 53)
        keys = torch.clamp(torch.searchsorted(zipf_cdf(n_keys, zipf, device), u), max=n_keys - 1)
    elif n_keys & (n_keys - 1) == 0:
        keys = hk & (n_keys - 1)
    else:
        keys = torch.remainder(_lsr(hk, 1), n_keys)
    ts = t0 + torch.div(i * 1000, rate, rounding_mode="floor")
    if ooo:
        ts = ts - torch.remainder(_lsr(splitmix64(i ^ 3), 1), ooo + 1)
    hv = splitmix64(i ^ seed_val)
    if value_type == "i64":
        vals = hv
    else:
        vals = _lsr(hv, 11).to(torch.float64) / float(1 << 53)
    return keys, ts, vals
