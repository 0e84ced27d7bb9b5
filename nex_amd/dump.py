"""Batched counterpart of the reference's `examples/dump.rs`: frames from a
capture file are parsed on the GPU a batch at a time (NEXG_OUT_RECORD) and
walked layer by layer with the per-protocol views of `nex_amd.views`,
printing what dump.rs:54-350 prints per frame.

    python -m nex_amd.dump capture.pcap [--batch N] [--limit N]
"""
import argparse
import sys
from typing import Iterator

import numpy as np

from . import abi
from .views import dump_records


def dump_capture(path: str, engine=None, batch_frames: int = 1 << 16, limit: int = 0) -> Iterator[str]:
    import torch

    from .engine import Engine, FrameBatch
    from .ingest import PcapReader
    eng = engine or Engine(0)
    rd = PcapReader(path)
    data = np.empty(batch_frames * 2048, np.uint8)
    offs = np.empty(batch_frames + 1, np.uint64)
    no = 1
    while True:
        n = rd.read_into(data, offs)
        if n == 0:
            break
        if limit:
            n = min(n, limit - no + 1)
        end = int(offs[n])
        frames = [bytes(data[int(offs[i]):int(offs[i + 1])]) for i in range(n)]
        dev = torch.from_numpy(data[:max(end, 16)].copy()).to(eng.torch_device)
        doffs = torch.from_numpy(offs[:n + 1].astype(np.int64)).to(eng.torch_device)
        recs = eng.parse_to_numpy(FrameBatch(data=dev, count=n, offsets=doffs), out_kind=abi.OUT_RECORD)
        yield from dump_records(recs, frames, path, no)
        no += n
        if limit and no > limit:
            break


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("capture", help="pcap / pcapng file")
    ap.add_argument("--batch", type=int, default=1 << 16, help="frames per GPU batch")
    ap.add_argument("--limit", type=int, default=0, help="stop after N frames")
    args = ap.parse_args(argv)
    for line in dump_capture(args.capture, batch_frames=args.batch, limit=args.limit):
        print(line)


if __name__ == "__main__":
    sys.exit(main())
