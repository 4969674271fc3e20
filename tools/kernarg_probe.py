"""Which launches make the HIP runtime issue a __amd_rocclr_copyBuffer (run under rocprofv3 --kernel-trace):
phases separated by torch.cuda.synchronize + a marker fill so the trace can be split."""
import os
import sys
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multimodal-image-transformer_amd"))
import native  # noqa: E402

dev = torch.device("cuda")
mark = torch.empty(1 << 20, device=dev)
R, d = 4032, 512
A = torch.randn(R, d, device=dev).to(torch.bfloat16)
B = torch.randn(R, d, device=dev).to(torch.bfloat16)
C = torch.empty(d, d, device=dev)
probs = [(A, B, C, d, d, R, d, d, None)]
ws = torch.empty((native.gemm_grouped_ws_bytes(probs) + 255) // 4, device=dev)
X = torch.randn(4096, 768, device=dev).to(torch.bfloat16)
W = torch.randn(768, 768, device=dev).to(torch.bfloat16)
Y = torch.empty(4096, 768, device=dev, dtype=torch.bfloat16)
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
evs = native.HipEvents(8)
tev = torch.cuda.Event()


def ev_hip():
    native.HipEvents.wait(s2.cuda_stream, evs.record(s1.cuda_stream))


def ev_hip_gemm():
    with torch.cuda.stream(s1):
        native.gemm(X, W, Y, 4096, 768, 768)
    native.HipEvents.wait(s2.cuda_stream, evs.record(s1.cuda_stream))
    with torch.cuda.stream(s2):
        native.gemm(X, W, Y, 4096, 768, 768)


for name, fn in [("ev_hip", ev_hip), ("ev_hip_gemm", ev_hip_gemm)]:
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    mark.fill_(1.0)
    torch.cuda.synchronize()
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    mark.fill_(2.0)
    torch.cuda.synchronize()
    print(name, "done", flush=True)
