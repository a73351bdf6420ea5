"""Chained (mipipe output feeds mipipe) stage comparison vs fp32 reference."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from mipipe.models import create_model
from mipipe.models.reference import ref_resnet
from mipipe.ops import kernels as K
import mipipe.nn as mnn


def cos(a, b):
    a, b = a.flatten().float(), b.flatten().float()
    return round((a @ b / (a.norm() * b.norm() + 1e-12)).item(), 5)


def nhwc(t):
    return t.permute(0, 2, 3, 1)


arch = sys.argv[1]
grad = len(sys.argv) > 2
torch.manual_seed(0)
m = create_model(arch, num_classes=100).cuda()
r = ref_resnet(arch, num_classes=100).cuda()
r.load_state_dict(m.state_dict())
x = torch.randn(16, 3, 64, 64, device="cuda")
for it in range(2):
    with torch.set_grad_enabled(grad):
        xm = K.nchw_to_nhwc(x, m.activation_dtype(x), 8)
        a = mnn.conv_bn_act(xm, m.conv1, m.bn1, relu=True)
        b = r.relu(r.bn1(r.conv1(x)))
        a = m.maxpool(a); b = r.maxpool(b)
        print(it, "stem+pool", cos(a, nhwc(b)), a.shape, a.stride(), a.dtype)
        for li in range(1, 5):
            for bi, (bm, br) in enumerate(zip(getattr(m, f"layer{li}"), getattr(r, f"layer{li}"))):
                a = bm(a); b = br(b)
                print(it, f"layer{li}.{bi}", cos(a, nhwc(b)), tuple(a.shape), a.stride(),
                      "absmax", float(a.float().abs().max()), float(b.abs().max()))
        pm = m.avgpool(a); pr = torch.flatten(r.avgpool(b), 1)
        print(it, "avgpool", cos(pm, pr), "fc", cos(m.fc(pm), r.fc(pr)))
