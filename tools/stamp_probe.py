"""Diagnostic: per-wave phase stamps of the fast query kernel (build with
-DCBN_STAMPS into libcbn_amd_stamps.so).  Prints median cycles per phase."""
import ctypes, os, sys, subprocess
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import continuousbayesiannetwork_amd._native as nat
nat.LIB_PATH = os.path.join(ROOT, "continuousbayesiannetwork_amd", "libcbn_amd_stamps.so")
from continuousbayesiannetwork_amd import BayesianNetwork
from helpers import chain_data, make_bn, sample_evidence

dev = torch.device("cuda:0")
lib = nat.load()
lib.cbn_debug_set_stamp_buffer.argtypes = [ctypes.c_void_p]
buf = torch.zeros(4096 * 16 * 8, dtype=torch.int64, device=dev)
data, cols, edges = chain_data(20, 32, 200000, 3, stay=0.8)
bn = make_bn(BayesianNetwork, edges, cols, data, device=dev)
ev = {k: torch.tensor(v, device=dev) for k, v in sample_evidence(data, cols, cols[:-1], 65536, 1000).items()}
for _ in range(20):
    bn.infer("X19", ev, N_max=32)
torch.cuda.synchronize()
nat.check(lib.cbn_debug_set_stamp_buffer(ctypes.c_void_p(buf.data_ptr())), "stamps")
buf.zero_()
bn.infer("X19", ev, N_max=32)   # stamps of the write pass overwrite the max pass's
torch.cuda.synchronize()
st = buf.view(-1, 8).cpu().numpy()
st = st[st[:, 0] > 0]
t0 = st[:, 0].min()
print("waves stamped:", len(st))
names = ["entry", "records built, fill issued", "sync (fill landed)", "ev loads issued", "offsets + wave exchange", "products", "store", "loop end"]
for k in range(8):
    v = st[:, k] - t0
    print(f"{k} {names[k]:28s} median {np.median(v):9.0f}  min {v.min():9.0f}  max {v.max():9.0f}  (cycles since first wave entry)")
for k in range(1, 8):
    d = st[:, k] - st[:, k - 1]
    print(f"  d{k} {names[k]:26s} median {np.median(d):9.0f}")
