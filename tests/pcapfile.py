"""TEST INFRASTRUCTURE ONLY: writers for classic pcap and pcapng files (the
published formats), used to exercise nex_amd.ingest / nexg_pcap_*."""
import struct


def classic(frames, ts=None, big_endian=False, nsec=False, linktype=1, snaplen=65535, caplens=None):
    e = ">" if big_endian else "<"
    magic = 0xA1B23C4D if nsec else 0xA1B2C3D4
    out = [struct.pack(e + "IHHiIII", magic, 2, 4, 0, 0, snaplen, linktype)]
    for i, f in enumerate(frames):
        t = ts[i] if ts else i * 1_000_001_000
        sec, frac = divmod(t, 10**9)
        if not nsec:
            frac //= 1000
        cap = len(f) if caplens is None else caplens[i]
        out.append(struct.pack(e + "IIII", sec, frac, cap, max(len(f), cap)) + f[:cap])
    return b"".join(out)


def _block(e, btype, body):
    body = body + b"\0" * ((-len(body)) % 4)
    n = 12 + len(body)
    return struct.pack(e + "II", btype, n) + body + struct.pack(e + "I", n)


def ng_shb(big_endian=False):
    e = ">" if big_endian else "<"
    return _block(e, 0x0A0D0D0A, struct.pack(e + "IHHq", 0x1A2B3C4D, 1, 0, -1))


def ng_idb(linktype=1, snaplen=0, tsresol=None, big_endian=False):
    e = ">" if big_endian else "<"
    opts = b""
    if tsresol is not None:
        opts = struct.pack(e + "HH", 9, 1) + bytes([tsresol]) + b"\0\0\0" + struct.pack(e + "HH", 0, 0)
    return _block(e, 1, struct.pack(e + "HHI", linktype, 0, snaplen) + opts)


def ng_epb(frame, ticks, iface=0, caplen=None, big_endian=False):
    e = ">" if big_endian else "<"
    cap = len(frame) if caplen is None else caplen
    return _block(e, 6, struct.pack(e + "IIIII", iface, ticks >> 32, ticks & 0xFFFFFFFF, cap, len(frame))
                  + frame[:cap])


def ng_spb(frame, big_endian=False):
    e = ">" if big_endian else "<"
    return _block(e, 3, struct.pack(e + "I", len(frame)) + frame)


def ng_opb(frame, ticks, iface=0, big_endian=False):
    e = ">" if big_endian else "<"
    return _block(e, 2, struct.pack(e + "HHIIII", iface, 0, ticks >> 32, ticks & 0xFFFFFFFF,
                                    len(frame), len(frame)) + frame)


def ng_nrb(big_endian=False):  # name resolution block: must be skipped
    e = ">" if big_endian else "<"
    return _block(e, 4, struct.pack(e + "HH", 0, 0))
