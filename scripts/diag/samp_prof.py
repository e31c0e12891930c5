"""One sampler launch (for rocprofv3 PMC runs): n = 10^4, 4096 graphs."""
import ctypes as ct, os, sys
sys.path.insert(0, os.getcwd())
import torch
from iib_project_ldpc_codes_amd import _native
L = _native.lib()
n, G = int(os.environ.get("N", "10000")), int(os.environ.get("G", "4096"))
chk = torch.empty((G, n * 3), dtype=torch.int32, device="cuda")
var = torch.empty_like(chk)
att = torch.empty(G, dtype=torch.int32, device="cuda")
assert L.ldpc_sample_regular_dev(n, 3, 6, 5, 0, G, chk.data_ptr(), var.data_ptr(), att.data_ptr(),
                                 torch.cuda.current_stream().cuda_stream) == 0
torch.cuda.synchronize()
print("mean attempts", att.float().mean().item())
