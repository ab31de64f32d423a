import sys, os, ctypes, struct
import numpy as np, torch
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))
from nghttp2_amd import workloads as W
L = ctypes.CDLL(os.path.join(HERE, "libdbg.so"))
vp = ctypes.c_void_p
L.nghttp2_amd_hd_huff_encode_batch.argtypes = [vp, vp, ctypes.c_uint32, vp, ctypes.c_size_t, vp, vp, ctypes.c_size_t, vp]
dev = torch.device("cuda:0")
pool, off = W.gen_pseudo_headers(1000)
n = len(off) - 1
src = torch.from_numpy(pool).to(dev); so = torch.from_numpy(off.view(np.int32)).to(dev)
dst = torch.zeros(200000, dtype=torch.uint8, device=dev); do = torch.zeros(n + 1, dtype=torch.int32, device=dev)
ws = torch.zeros(1 << 20, dtype=torch.uint8, device=dev)
rv = L.nghttp2_amd_hd_huff_encode_batch(vp(src.data_ptr()), vp(so.data_ptr()), n, vp(dst.data_ptr()), 200000, vp(do.data_ptr()), vp(ws.data_ptr()), 1 << 20, None)
torch.cuda.synchronize()
buf = (ctypes.c_uint32 * (64 * 8))()
L.nghttp2_amd_hd__encdbg(buf)
d = np.array(buf).reshape(64, 8)
print("rv", rv, "off", off[:6].tolist())
for l in range(8):
    print(l, "start", d[l,0], "sidx", d[l,1], "S", d[l,2], "Pme", d[l,3], "hm", hex(d[l,4]), "vm", hex(d[l,5]), "anchor", d[l,6], "bits", d[l,7])
