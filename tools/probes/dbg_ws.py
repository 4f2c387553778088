import ctypes as C, sys, torch
sys.path.insert(0, '.')
from optical_flow_amd import _lib, ops
from optical_flow_amd._lib import ACT_LEAKY, ACT_NONE, call
lib = _lib.lib()
n, h, w, cin, cout = 8, 128, 256, 128, int(sys.argv[1]) if len(sys.argv) > 1 else 96
torch.manual_seed(0)
x = torch.randn(n, h, w, cin, device="cuda")
wt = torch.randn(3, 3, cin, cout, device="cuda") * 0.05
b = torch.zeros(cout, device="cuda")
outs = {}
for form in (2, 0):
    lib.of_set_tuning(12, form)
    layer = ops.ConvLayer(wt, b, act=ACT_NONE, cin_p=cin, precision="bf16")
    d = layer.desc(n, h, w)
    wf, wd = layer.packed(d)
    fent, fws = layer.fwd_entry(d)
    ws = torch.empty(fws // 4 + 4, device="cuda")
    y = torch.full((n, h, w, cout), 7.0, device="cuda")
    call(fent, C.byref(d), ops._ptr(x), cin, ops._ptr(wf), ops._ptr(b), None, None, None, None, 1e-3, None, 0,
         ACT_NONE, 0.3, None, 0, ops._ptr(y), cout, ops._ptr(ws), fws, ops._stream())
    torch.cuda.synchronize()
    outs[form] = y
e = (outs[2] - outs[0]).abs()
bad = e > 1e-3 * outs[0].abs().max()
print("bad frac", bad.float().mean().item())
print("by channel", bad.float().mean(dim=(0, 1, 2)).cpu().numpy().round(2))
by_oy = bad.float().mean(dim=(0, 2, 3)).reshape(-1, 8).mean(0)
by_ox = bad.float().mean(dim=(0, 1, 3)).reshape(-1, 32).mean(0)
print("by oy%8", by_oy.cpu().numpy().round(2))
print("by ox%32", by_ox.cpu().numpy().round(2))
print("unwritten (7.0)", (outs[2] == 7.0).float().mean().item())
