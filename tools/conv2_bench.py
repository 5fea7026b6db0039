import os, sys
sys.path.insert(0, "/root/repo/asr-transformer_amd"); sys.path.insert(0, "/root/repo")
import torch
from asrx import kernels as K
from bench import _graph_time_ms
B, F1, T1 = 64, 39, 499
F2, T2 = 19, 249
g = torch.Generator(device="cuda").manual_seed(0)
y1 = torch.relu(torch.randn(B, F1, T1, 64, device="cuda", generator=g)).bfloat16()
w2 = (torch.randn(64, 576, device="cuda", generator=g) * 0.05).bfloat16()
b2 = torch.randn(64, device="cuda", generator=g)
M = B * T2 * F2
out = torch.empty(M, 64, device="cuda", dtype=torch.bfloat16)
cols = torch.empty(M, 576, device="cuda", dtype=torch.bfloat16)
out2 = torch.empty_like(out)
def old():
    K.im2col_conv2(y1, cols)
    K.gemm(cols, w2, out2, M, 64, 576, lda=576, ldb=576, ldc=64, bias=b2, relu=True)
old(); K.conv2_fwd(y1, w2, b2, out); torch.cuda.synchronize()
print("maxdiff", float((out.float() - out2.float()).abs().max()), float(out2.float().abs().max()))
print("implicit %.1f us" % (_graph_time_ms(lambda: K.conv2_fwd(y1, w2, b2, out), launches=10) * 1e3))
print("im2col+gemm %.1f us" % (_graph_time_ms(old, launches=10) * 1e3))
dy2 = (torch.randn(M, 64, device="cuda", generator=g) * 0.1).bfloat16()
dw = torch.zeros(64, 576, device="cuda"); db = torch.zeros(64, device="cuda")
dw2 = torch.zeros(64, 576, device="cuda"); db2 = torch.zeros(64, device="cuda")
K.im2col_conv2(y1, cols)
K.conv2_wgrad(dy2, y1, dw, db)
K.linear_wgrad(dy2, cols, dw2, bias_grad=db2)
torch.cuda.synchronize()
print("wgrad maxdiff", float((dw - dw2).abs().max()), float(dw2.abs().max()), float((db - db2).abs().max()))
print("wgrad gather %.1f us" % (_graph_time_ms(lambda: K.conv2_wgrad(dy2, y1, dw, db), launches=10) * 1e3))
print("wgrad cols %.1f us" % (_graph_time_ms(lambda: K.linear_wgrad(dy2, cols, dw2, bias_grad=db2), launches=10) * 1e3))
