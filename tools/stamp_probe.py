"""Diagnostic: per-wave phase stamps of the fast query kernel (build with
-DCBN_STAMPS into libcbn_amd_stamps.so).  Prints median cycles per phase."""
import ctypes, os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import continuousbayesiannetwork_amd._native as nat
nat.LIB_PATH = os.environ.get("CBN_LIB_PATH") or os.path.join(ROOT, "continuousbayesiannetwork_amd",
                                                               "libcbn_amd_stamps.so")
from continuousbayesiannetwork_amd import BayesianNetwork
from helpers import chain_data, make_bn, sample_evidence

dev = torch.device("cuda:0")
lib = nat.load()
lib.cbn_debug_set_stamp_buffer.argtypes = [ctypes.c_void_p]
S = 12
buf = torch.zeros(4096 * 16 * S, dtype=torch.int64, device=dev)
if os.environ.get("GRID"):  # BASELINE configs[4]: peaked 10 x 10 grid, k_query_fast on global tables
    from helpers import grid_data
    data, cols, edges = grid_data(400_000, 3, side=10, d=64, keep=0.995, noise=0)
    target, Q, NM = "X99", 65536, 64
elif os.environ.get("ALARM"):  # BASELINE configs[2]: k_query_fast on global tables (tools/bench_alarm.py)
    from helpers import alarm_like_data
    data, cols, edges = alarm_like_data(200_000, 5)
    target, Q, NM = "X35", 262144, 8
else:  # configs[1]: the staged kernel
    data, cols, edges = chain_data(20, 32, 200000, 3, stay=0.8)
    target, Q, NM = "X19", 65536, 32
bn = make_bn(BayesianNetwork, edges, cols, data, device=dev)
bn.engine.fused = os.environ.get("TWO_PASS") is None
names_ev = [c for c in cols if c != target]
evs = []
for b in range(8):
    evs.append({k: torch.tensor(v, device=dev) for k, v in sample_evidence(data, cols, names_ev, Q, 1000 + b).items()})
for i in range(40):
    bn.infer(target, evs[i % 8], N_max=NM)
torch.cuda.synchronize()
nat.check(lib.cbn_debug_set_stamp_buffer(ctypes.c_void_p(buf.data_ptr())), "stamps")
buf.zero_()
bn.infer(target, evs[3], N_max=NM)
torch.cuda.synchronize()
st = buf.view(-1, S).cpu().numpy()
st = st[st[:, 0] > 0]
print("waves stamped:", len(st), "fused" if bn.engine.fused else "two-pass (write pass stamps)")
names = ["entry", "kernargs + fill issued + ptab", "sync (fill landed)", "ev loads issued", "offsets + wave exchange",
         "products", "store/acc", "loop end", "barrier passed (tid0)", "block sync after barrier", "stored"]
for k in range(1, 11):
    ok = (st[:, k] > 0) & (st[:, k - 1] > 0)
    if ok.sum() == 0:
        continue
    d = st[ok, k] - st[ok, k - 1]
    print(f"  d{k:<2} {names[k]:28s} median {np.median(d):9.0f}  p90 {np.percentile(d, 90):9.0f}  max {d.max():9.0f}")
tot = st[:, 10] - st[:, 0] if bn.engine.fused else st[:, 7] - st[:, 0]
tot = tot[tot > 0]
if tot.size == 0:  # (no post-barrier stamps: entry -> loop end)
    tot = st[:, 7] - st[:, 0]
    tot = tot[tot > 0]
print("  total per wave: median", np.median(tot), "max", tot.max(), "(units: 10 ns ticks of s_memrealtime)")
# launch / arrival skew within each XCD (blocks b and b+8 share an XCD, so their s_memtime is comparable)
full = buf.view(-1, 16, S).cpu().numpy()  # [block, wave, stamp]
nb = int((full[:, 0, 0] > 0).sum())
e = np.array([full[b, :, 0].min() for b in range(nb)])
a = np.array([full[b, :, 7].max() for b in range(nb)])
t0 = e.min()
print("block entry (ticks after first): p50 %d p90 %d max %d" % tuple(np.percentile(e - t0, [50, 90, 100])))
print("block arrival at barrier:        p50 %d p90 %d max %d" % tuple(np.percentile(a - t0, [50, 90, 100])))
print("per-block entry->arrival:        p50 %d p90 %d max %d" % tuple(np.percentile(a - e, [50, 90, 100])))
late = np.argsort(e)[-8:]
print("latest-entering blocks:", late.tolist(), (e[late] - t0).tolist())
grp = np.array([e[b::8].min() - t0 for b in range(8)])
print("first block entry per b % 8 group:", grp.tolist())
# prologue by wave role (staged kernel: waves 0..3 issue the image DMA, 4..15 stage the evidence)
for name, ws in (("DMA waves 0-3", slice(0, 4)), ("evidence waves 4-15", slice(4, 16))):
    sub = full[:nb, ws, :].reshape(-1, S)
    parts = []
    for k in (1, 2, 3):
        d = sub[:, k] - sub[:, k - 1]
        parts.append(f"d{k} p50 {np.median(d):.0f} p90 {np.percentile(d, 90):.0f}")
    print(f"  {name:20s}", " | ".join(parts), f"| entry->sync p50 {np.median(sub[:, 3] - sub[:, 0]):.0f}")
