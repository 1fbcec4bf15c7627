"""Root-merge cost at the 8-GPU exchange shape (tooling): P = 8 rank lists x 1000 queries x
k = 10, merged by bsr_global_top_k on the device (k_merge_lists) and on the host
(merge_top_k_lists), results compared.  Run under rocprofv3 --kernel-trace --stats for the
kernel's own duration."""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, "better-search-rag-rust_amd")
import bsr  # noqa: E402

P, Q, K = 8, 1000, 10
rng = np.random.default_rng(3)
ld = np.sort(rng.random((P, Q, K), dtype=np.float32), axis=2)
li = (np.arange(P, dtype=np.uint64)[:, None, None] * 1_250_000 + rng.integers(0, 1_250_000, (P, Q, K)).astype(np.uint64))
lc = np.full((P, Q), K, np.uint32)
d_i, d_d, d_c = (torch.from_numpy(li.view(np.int64)).cuda(), torch.from_numpy(ld).cuda(),
                 torch.from_numpy(lc.view(np.int32)).cuda())
o_i = torch.empty((Q, K), dtype=torch.int64, device="cuda")
o_d = torch.empty((Q, K), dtype=torch.float32, device="cuda")
o_c = torch.empty(Q, dtype=torch.int32, device="cuda")
lib = bsr.lib()


def dev_merge():
    st = lib.bsr_global_top_k(d_i.data_ptr(), d_d.data_ptr(), d_c.data_ptr(), P, Q, K, K, o_i.data_ptr(),
                              o_d.data_ptr(), o_c.data_ptr())
    assert st == 0


for _ in range(5):
    dev_merge()
torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(50):
    dev_merge()
torch.cuda.synchronize()
dev_ms = (time.perf_counter() - t) / 50 * 1e3
hi, hd, hc = bsr.merge_top_k_lists(li, ld, lc, K)
t = time.perf_counter()
for _ in range(20):
    bsr.merge_top_k_lists(li, ld, lc, K)
host_ms = (time.perf_counter() - t) / 20 * 1e3
same = (np.array_equal(o_i.cpu().numpy().view(np.uint64), hi) and np.array_equal(o_c.cpu().numpy().view(np.uint32), hc)
        and np.array_equal(o_d.cpu().numpy().view(np.uint32), hd.view(np.uint32)))
print(f"P={P} Q={Q} k={K}: device merge call {dev_ms:.3f} ms (incl. its NaN-word readback), host merge {host_ms:.3f} ms, "
      f"identical={same}")
