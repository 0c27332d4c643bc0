# Debug: slice 5 of test_deshred_batch_matches_oracle through the individual stages.
import random, sys
sys.path[:0] = ['.', 'oracle', 'tests']
import numpy as np, torch
import ed25519_oracle as ed, rs_oracle as o, shredder_oracle as so, slice_oracle as sl, shred_wire_oracle as wire
from alpenglow_amd import rs
import test_shredder_pipeline as T
torch.zeros(1, device='cuda:0')
ctx = rs.Context(0)
dev = torch.device('cuda:0')
rng = random.Random(77)
slices = T._slices(rng, 9, 1024)
clean = [so.shred(p, d, slot, si, last, T.SEED) for p, d, slot, si, last in slices]
for b, cnt in ((1, 32), (2, 31), (3, 40)):
    rng.sample(range(64), cnt)
payload5 = b"\x07" + bytes(rng.randrange(256) for _ in range(32700))
raw5 = o.coder_shred(payload5, 32)
rows5, root5, sig5 = so.datagrams(raw5.data, raw5.coding, slices[5][2], slices[5][3], slices[5][4], T.SEED)
print("payload5 len", len(payload5), "S", len(raw5.data[0]), "pkt len", len(rows5[0]))
d = wire.deserialize(rows5[0]); print("deser ok", d is not None, d[0], d[4], len(d[5]), len(d[7]))
pk = ed.secret_to_public(T.SEED)
print("oracle verify", ed.verify(pk, ed.slice_commitment(slices[5][2], slices[5][3], slices[5][4], root5), sig5))
inp = [[None] * 64 for _ in range(9)]
inp[5] = rows5
inp[0] = clean[0][0]
res, out, cw = T._deshred(ctx, dev, inp, T._dev(np.frombuffer(pk, np.uint8), dev), 1024)
print("status", res.status.tolist())
