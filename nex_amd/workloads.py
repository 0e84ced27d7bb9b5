"""The SURVEY.md Appendix C malformed mix, for measuring the parse path's
fallback cost (bench.py --workload malformed).

Frames start as the IMIX generator's (nexg_gen_frames on the device), then
half of them get one structural mutation, drawn and applied with vectorised
numpy on the host so the mix is deterministic (seeded) and fast to build:
truncation, Ethernet padding, a random IPv4 total length / IPv6 payload
length, a random version/IHL byte, random UDP / TCP length fields, an IPv6
hop-by-hop header, an 802.1Q tag, IP protocol 200 (-> Reserved), or random
bytes. Mutated frames leave the canonical fast paths and run the generic
parse core on the GPU; the result is a packed batch (offsets only).
"""
import numpy as np

from . import abi

MUTATIONS = ("truncate", "pad", "ip_length", "ver_ihl", "l4_length", "ipv6_hbh", "vlan", "proto200", "random")
#: not in the App. C mix; selectable through `kinds` (tools/bench_malformed.py):
#: real-traffic TCP option lists inserted after the TCP header of a TCP frame
#: (data offset and IP length grown to fit, checksums left stale):
#: tcp_ts = NOP NOP Timestamps (12 B, data offset 8: most data segments),
#: tcp_sack = NOP NOP SACK with 1-4 blocks (12-36 B), tcp_mss = MSS alone (4 B, SYN-ACK)
EXTRA = ("tcp_ts", "tcp_sack", "tcp_mss")
_ALL = MUTATIONS + EXTRA


def malformed_mix(engine, count: int, seed: int = abi.DEFAULT_SEED, mutate_share: float = 0.5,
                  kinds=MUTATIONS):
    """(FrameBatch on the engine's device, dict of per-mutation counts);
    `kinds` restricts the mutations drawn (tools/bench_malformed.py)."""
    import torch

    from .engine import FrameBatch
    base = engine.gen_batch(abi.WL_IMIX, count, seed=seed)
    torch.cuda.synchronize(engine.torch_device)
    offs = base.offsets.cpu().numpy().astype(np.int64)
    data = base.data.cpu().numpy()[: offs[-1]]
    out, new_offs, counts = mutate_packed(data, offs, seed, mutate_share, kinds)
    dev = torch.from_numpy(np.concatenate([out, np.zeros(16, np.uint8)])).to(engine.torch_device)
    doffs = torch.from_numpy(new_offs).to(engine.torch_device)
    return FrameBatch(data=dev[: int(new_offs[-1])], count=count, offsets=doffs), counts


def mutate_packed(data, offs, seed: int = abi.DEFAULT_SEED, mutate_share: float = 0.5, kinds=MUTATIONS):
    """The mutations of malformed_mix on a host packed batch (bytes, count+1
    offsets): (mutated bytes, new offsets, dict of per-mutation counts)."""
    count = len(offs) - 1
    lens = np.diff(offs)
    rng = np.random.default_rng(seed)
    pick = np.array([_ALL.index(k) for k in kinds])
    kind = np.where(rng.random(count) < mutate_share, pick[rng.integers(0, len(pick), count)], -1)
    # per-frame byte edits on a copy of the frame bytes (lengths unchanged)
    buf = data.copy()
    eth_v4 = (buf[offs[:-1] + 12] == 0x08) & (buf[offs[:-1] + 13] == 0x00)
    sel = lambda k: np.nonzero(kind == _ALL.index(k))[0]
    i = sel("ip_length")  # bytes 16..17 (IPv4 total length) / 18..19 (IPv6 payload length)
    pos = offs[i] + np.where(eth_v4[i], 16, 18)
    v = rng.integers(0, 1 << 16, len(i))
    buf[pos], buf[pos + 1] = v >> 8, v & 0xFF
    i = sel("ver_ihl")
    buf[offs[i] + 14] = rng.integers(0, 256, len(i))
    i = sel("l4_length")  # UDP length / TCP data offset / ICMP type area of a v4 or v6 frame
    l4 = offs[i] + np.where(eth_v4[i], 34, 54)
    v4b, v12 = rng.integers(0, 256, len(i)), rng.integers(0, 256, len(i))
    end = offs[i + 1]  # a 64-B IPv6/UDP frame ends at byte 62 + 2: byte l4 + 12 is past it
    buf[l4 + 4] = np.where(l4 + 4 < end, v4b, buf[np.minimum(l4 + 4, len(buf) - 1)])
    k = l4 + 12 < end
    buf[l4[k] + 12] = v12[k]
    i = sel("proto200")
    buf[offs[i] + np.where(eth_v4[i], 23, 20)] = 200
    i = sel("random")
    for j in i:  # few enough frames to fill one at a time
        buf[offs[j]:offs[j + 1]] = rng.integers(0, 256, lens[j], dtype=np.uint8)
    # length-changing mutations: new lengths + inserted / appended bytes
    new_len = lens.copy()
    i = sel("truncate")
    new_len[i] = (rng.random(len(i)) * lens[i]).astype(np.int64)
    pad = np.zeros(count, np.int64)
    i = sel("pad")
    pad[i] = rng.integers(1, 64, len(i))
    ins = np.zeros(count, np.int64)  # bytes inserted after byte 13 (VLAN) / 54 (IPv6 HBH)
    ins[sel("vlan")] = 4
    hbh = sel("ipv6_hbh")
    hbh = hbh[~eth_v4[hbh]]
    ins[hbh] = 8
    topt = {}  # frame -> TCP option bytes inserted after its 20-B TCP header
    for k in ("tcp_ts", "tcp_sack", "tcp_mss"):
        t = sel(k)
        t = t[buf[offs[t] + np.where(eth_v4[t], 23, 20)] == 6]
        blocks = rng.integers(1, 5, len(t))
        body = rng.integers(0, 256, (len(t), 32), dtype=np.uint8)
        for j, nb, b in zip(t.tolist(), blocks.tolist(), body):
            if k == "tcp_ts":
                topt[j] = np.concatenate([np.array([1, 1, 8, 10], np.uint8), b[:8]])
            elif k == "tcp_sack":
                topt[j] = np.concatenate([np.array([1, 1, 5, 2 + 8 * nb], np.uint8), b[:8 * nb]])
            else:
                topt[j] = np.array([2, 4, 5, 180], np.uint8)
            ins[j] = len(topt[j])
    new_len = new_len + pad + ins
    new_offs = np.zeros(count + 1, np.int64)
    np.cumsum(new_len, out=new_offs[1:])
    out = np.zeros(int(new_offs[-1]), np.uint8)
    plain = np.nonzero((ins == 0) & (pad == 0))[0]
    # frames without inserts: gathers of their (possibly truncated) bytes, in
    # chunks so the index arrays stay small (one rank per GPU builds its mix)
    for c0 in range(0, len(plain), 1 << 16):
        sel = plain[c0:c0 + (1 << 16)]
        ramp = _ramp(new_len[sel])
        out[np.repeat(new_offs[:-1][sel], new_len[sel]) + ramp] = buf[np.repeat(offs[:-1][sel], new_len[sel]) + ramp]
    for j in np.nonzero((ins != 0) | (pad != 0))[0]:  # the frames the gathers above left out
        f = buf[offs[j]:offs[j + 1]]
        if pad[j]:
            f = np.concatenate([f, rng.integers(0, 256, pad[j], dtype=np.uint8)])
        elif j in topt:  # TCP options after the TCP header, data offset grown to fit
            o = topt[j]
            l4 = 34 if eth_v4[j] else 54
            g = f.copy()
            g[l4 + 12] = ((5 + len(o) // 4) << 4) | (g[l4 + 12] & 0x0F)
            k = 16 if eth_v4[j] else 18
            v = (((int(g[k]) << 8) | int(g[k + 1])) + len(o)) & 0xFFFF  # u16 field: wraps
            g[k], g[k + 1] = v >> 8, v & 0xFF
            f = np.concatenate([g[:l4 + 20], o, g[l4 + 20:]])
        elif ins[j] == 4:  # 802.1Q tag in front of the EtherType (frame[12:14])
            f = np.concatenate([f[:12], np.array([0x81, 0, 0, 0x64], np.uint8), f[12:]])
        elif ins[j] == 8:  # hop-by-hop header carrying the original next header
            nh = f[20]
            g = f.copy()
            g[20] = 0
            pl = (((int(g[18]) << 8) | int(g[19])) + 8) & 0xFFFF  # u16 field: wraps
            g[18], g[19] = pl >> 8, pl & 0xFF
            f = np.concatenate([g[:54], np.array([nh, 0, 0, 0, 0, 0, 0, 0], np.uint8), g[54:]])
        out[new_offs[j]:new_offs[j] + len(f)] = f
    counts = {m: int((kind == k).sum()) for k, m in enumerate(_ALL) if m in kinds}
    counts["unmodified"] = int((kind < 0).sum())
    return out, new_offs, counts


def _ramp(lengths):
    """[0..l0), [0..l1), ... concatenated (vectorised)."""
    total = int(lengths.sum())
    if total == 0:
        return np.zeros(0, np.int64)
    starts = np.repeat(np.cumsum(lengths) - lengths, lengths)
    return np.arange(total, dtype=np.int64) - starts


def tiled(batch, times: int):
    """The packed batch repeated `times` times back to back on its device
    (the bench's full-size malformed batch from a 1M-frame mix)."""
    import torch

    from .engine import FrameBatch
    n, span = batch.count, int(batch.offsets[batch.count].item())
    # one allocation for the result, filled in place (repeat + cat made two
    # full-size allocations, the batch living in the second)
    buf = torch.zeros(times * span + 16, dtype=batch.data.dtype, device=batch.data.device)
    for k in range(times):
        buf[k * span:(k + 1) * span].copy_(batch.data[:span])
    base = batch.offsets[:n]
    offs = torch.cat([base + k * span for k in range(times)] +
                     [torch.tensor([times * span], dtype=base.dtype, device=base.device)])
    return FrameBatch(data=buf[: times * span], count=n * times, offsets=offs)


#: the real-traffic TCP option shapes of tcp.rs:731-836 timed in bench.py's
#: `real_traffic` object: 70 % of the IMIX's TCP segments carry one of them
REAL_TRAFFIC_KINDS = EXTRA
REAL_TRAFFIC_SHARE = 0.7


def real_traffic(engine, count: int, seed: int = abi.DEFAULT_SEED, fix_checksums: bool = True):
    """IMIX whose TCP segments carry the option lists of real traffic
    (timestamps, SACK blocks, MSS; `malformed_mix` kinds tcp_ts / tcp_sack /
    tcp_mss at REAL_TRAFFIC_SHARE), with the IP and L4 checksums made valid
    again on the device by nexg_recompute_checksums_batch (the mutable views'
    recompute_checksum, ipv4.rs:669-679 / tcp.rs:1009-1040), as a capture of
    healthy traffic would hold them. (FrameBatch, per-kind counts)."""
    import torch
    batch, counts = malformed_mix(engine, count, seed=seed, mutate_share=REAL_TRAFFIC_SHARE,
                                  kinds=REAL_TRAFFIC_KINDS)
    if fix_checksums:
        engine.recompute_checksums(batch, report=False)
        torch.cuda.synchronize(engine.torch_device)
    return batch, counts
