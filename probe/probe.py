import ctypes, torch, os
lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libprobe.so"))
A = torch.randn(16, 4, device="cuda"); B = torch.randn(4, 16, device="cuda"); C = torch.empty(16, 16, device="cuda")
s = torch.cuda.current_stream().cuda_stream
rc = lib.probe_mfma(ctypes.c_void_p(A.data_ptr()), ctypes.c_void_p(B.data_ptr()), ctypes.c_void_p(C.data_ptr()), ctypes.c_void_p(s))
torch.cuda.synchronize()
print("rc", rc, "maxerr", (C - A @ B).abs().max().item())
maps = open("/proc/self/maps").read()
print("hip runtimes:", sorted({l.split()[-1] for l in maps.splitlines() if "amdhip64" in l}))
g = torch.cuda.CUDAGraph()
C2 = torch.zeros_like(C)
with torch.cuda.graph(g):
    lib.probe_mfma(ctypes.c_void_p(A.data_ptr()), ctypes.c_void_p(B.data_ptr()), ctypes.c_void_p(C2.data_ptr()), ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
g.replay(); torch.cuda.synchronize()
print("graph maxerr", (C2 - A @ B).abs().max().item())
print(torch.cuda.get_device_name(0), os.cpu_count())
