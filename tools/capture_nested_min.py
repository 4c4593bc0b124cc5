"""Minimal HIP-graph capture with a NESTED fork (capture stream -> side A -> side B, joined back
B -> A -> capture stream) in plain torch, no dsvt code: does capture_end survive it?
usage: python tools/capture_nested_min.py MODE   (MODE: noalloc | alloc | allocfree | flat)"""
import faulthandler
import sys

import torch

faulthandler.enable()
mode = sys.argv[1] if len(sys.argv) > 1 else "alloc"
dev = torch.device("cuda")
A, B = torch.cuda.Stream(), torch.cuda.Stream()
x = torch.ones(1 << 20, device=dev)
buf = torch.zeros_like(x)


def body():
    cur = torch.cuda.current_stream()
    A.wait_stream(cur)
    with torch.cuda.stream(A):
        y = x * 2
        if mode == "flat":
            buf.copy_(y + 1)
        else:
            B.wait_stream(A)
            with torch.cuda.stream(B):
                if mode == "noalloc":
                    buf.add_(1)
                else:
                    z = y + 1            # allocated on B inside the capture
                    buf.copy_(z)
                    if mode == "allocfree":
                        del z
            A.wait_stream(B)
        buf.add_(y)
    cur.wait_stream(A)


s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    body()
torch.cuda.current_stream().wait_stream(s)
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
print(mode, "capturing", flush=True)
with torch.cuda.graph(g):
    body()
print(mode, "captured", flush=True)
g.replay()
torch.cuda.synchronize()
print(mode, "replayed", buf[:2].tolist(), flush=True)
