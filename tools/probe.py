"""GPU-box probe: HIP runtime sharing between torch and an in-tree hipcc .so,
MFMA 16x16x32 bf16 operand layout check, and device properties."""
import ctypes, os, subprocess, sys, time
import torch

here = os.path.dirname(os.path.abspath(__file__))
so = os.path.join(here, "libprobe.so")
if not os.path.exists(so):
    subprocess.check_call(["hipcc", "-O3", "--offload-arch=gfx950", "-fPIC", "-shared",
                           os.path.join(here, "probe_kernel.hip"), "-o", so])
print("torch", torch.__version__, "hip", torch.version.hip, "cuda avail", torch.cuda.is_available())
p = torch.cuda.get_device_properties(0)
print("device", p.name, "CUs", p.multi_processor_count, "mem GB", p.total_memory / 1e9, getattr(p, "gcnArchName", ""))
lib = ctypes.CDLL(so)
x = torch.zeros(1000, device="cuda")
s = torch.cuda.current_stream().cuda_stream
rc = lib.launch_add1(ctypes.c_void_p(x.data_ptr()), 1000, ctypes.c_void_p(s))
torch.cuda.synchronize()
print("add1 rc", rc, "sum", x.sum().item())
A = torch.randint(-4, 5, (16, 32)).float()
B = torch.randint(-4, 5, (32, 16)).float()
C = torch.zeros(16, 16, device="cuda")
Ab = A.bfloat16().cuda().contiguous(); Bb = B.bfloat16().cuda().contiguous()
lib.launch_mfma(ctypes.c_void_p(Ab.data_ptr()), ctypes.c_void_p(Bb.data_ptr()), ctypes.c_void_p(C.data_ptr()), ctypes.c_void_p(s))
torch.cuda.synchronize()
print("mfma max err", (C.cpu() - A @ B).abs().max().item())
# graph capture of ctypes launch
g = torch.cuda.CUDAGraph()
y = torch.zeros(1000, device="cuda")
st = torch.cuda.Stream()
with torch.cuda.stream(st):
    with torch.cuda.graph(g):
        lib.launch_add1(ctypes.c_void_p(y.data_ptr()), 1000, ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
for _ in range(3):
    g.replay()
torch.cuda.synchronize()
print("graph replay sum (expect 3000)", y.sum().item())
a = torch.randn(8192, 512, device="cuda", dtype=torch.bfloat16)
w = torch.randn(1536, 512, device="cuda", dtype=torch.bfloat16)
for shape in [(8192, 512, 1536), (8192, 512, 512), (8192, 1024, 512), (8192, 512, 1024), (8192, 512, 10000)]:
    M, K, N = shape
    a = torch.randn(M, K, device="cuda", dtype=torch.bfloat16); w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)
    for _ in range(3): torch.nn.functional.linear(a, w)
    torch.cuda.synchronize(); t = time.time()
    for _ in range(50): torch.nn.functional.linear(a, w)
    torch.cuda.synchronize(); dt = (time.time() - t) / 50
    print(f"hipblaslt linear M{M} K{K} N{N}: {dt*1e6:.1f} us  {2*M*N*K/dt/1e12:.0f} TF")
