"""Diagnostic: batched vs per-frame vs oracle on the bench sequence (first frames)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
import dvc_amd, oracle
from tests.test_bench_config import _sequence

W, H = 1920, 1080
dev = torch.device("cuda", 0)
for batch in [int(a) for a in sys.argv[1:]] or [383]:
    ring, idx, seq, first = _sequence(W, H, batch + 1 if batch > 8 else 64, False, 0, dev)
    n = 8
    ovb = torch.empty_like(seq); cpb = torch.empty_like(seq)
    wb = dvc_amd.FDWorker(W, H, device_ptrs=True, max_batch=batch)
    wb.prime(first); wb.step_batch(seq, ovb, cpb); wb.sync()
    wf = dvc_amd.FDWorker(W, H, device_ptrs=True)
    wf.prime(first)
    ref = oracle.OracleFD(W, H); ref.prime(ring[0])
    ov = torch.empty_like(seq[0]); cp = torch.empty_like(seq[0])
    for k in range(n):
        wf.step(seq[k], ov, cp)
        rov, rcp, racc = ref.step(ring[idx[k]])
        a = ovb[k].cpu().numpy(); b = ov.cpu().numpy()
        c = cpb[k].cpu().numpy(); d = cp.cpu().numpy()
        print(f"batch {batch} frame {k}: ov b!=f {(a!=b).any(-1).sum()} b!=o {(a!=rov).any(-1).sum()} f!=o {(b!=rov).any(-1).sum()} | "
              f"cp b!=f {(c!=d).any(-1).sum()} b!=o {(c!=rcp).any(-1).sum()} f!=o {(d!=rcp).any(-1).sum()}", flush=True)
        if (a != b).any():
            ys, xs = np.nonzero((a != b).any(-1))
            print("   first diffs", list(zip(ys[:5].tolist(), xs[:5].tolist())), "bbox", ys.min(), ys.max(), xs.min(), xs.max())
    wb.close(); wf.close(); ref.close()
