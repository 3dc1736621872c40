#!/usr/bin/env python
"""Which hardware CUs does a CU-masked stream use?  Prints distinct (xcc, se, sh, cu) per mask."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from gsc_amd.native import load
    nat = load()
    n = nat.cu_count()
    out = torch.zeros(4096, dtype=torch.int32, device="cuda")

    def probe(cus, label):
        s = torch.cuda.ExternalStream(nat.create_cu_masked_stream(cus)) if cus is not None else torch.cuda.current_stream()
        out.zero_()
        nat.cu_probe(out.data_ptr(), 4096, 200000, s.cuda_stream)
        torch.cuda.synchronize()
        v = out.cpu().tolist()
        ids = set()
        for x in v:
            xcc, hw = x >> 16, x & 0xffff
            cu, sh, se = hw & 0xf, (hw >> 4) & 1, (hw >> 5) & 0x7
            ids.add((xcc, se, sh, cu))
        xccs = sorted({i[0] for i in ids})
        per = {x: sum(1 for i in ids if i[0] == x) for x in xccs}
        print(f"{label:>28}: {len(ids):3d} distinct CUs  per-XCC {per}", flush=True)
        return ids

    probe(None, "default stream")
    probe(list(range(n)), "all bits")
    probe(list(range(32)), "bits 0-31")
    probe(list(range(64)), "bits 0-63")
    probe([i for i in range(n) if i % 8 == 0], "bits i%8==0")
    probe([i for i in range(n) if i % 4 == 0], "bits i%4==0")
    probe([i for i in range(n) if i % 8 in (0, 1)], "bits i%8 in {0,1}")
    probe(list(range(128)), "bits 0-127")
    probe(list(range(128, 256)), "bits 128-255")
    # per-bit mapping (mask bit -> xcc, se, sh, cu) for the first 64 bits
    for i in range(64):
        ids = probe([i], f"bit {i}")
        print(f"    bit {i} -> {sorted(ids)}", flush=True)


if __name__ == "__main__":
    main()
