"""Stage-by-stage comparison of mipipe ResNet (bf16 HIP path) vs the plain-torch fp32 model."""
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


arch = sys.argv[1] if len(sys.argv) > 1 else "resnet18"
torch.manual_seed(0)
m = create_model(arch, num_classes=100).cuda()
r = ref_resnet(arch, num_classes=100).cuda()
r.load_state_dict(m.state_dict())
x = torch.randn(16, 3, 64, 64, device="cuda")
with torch.no_grad():
    xm = K.nchw_to_nhwc(x, m.activation_dtype(x), 8)
    a = mnn.conv_bn_act(xm, m.conv1, m.bn1, relu=True)
    b = r.relu(r.bn1(r.conv1(x)))
    print("stem", cos(a, nhwc(b)))
    # isolate: feed identical input into each stage
    a2 = m.maxpool(a); b2 = r.maxpool(b); print("maxpool", cos(a2, nhwc(b2)))
    cur_ref = b2
    for li in range(1, 5):
        lm, lr = getattr(m, f"layer{li}"), getattr(r, f"layer{li}")
        inp = nhwc(cur_ref).contiguous().to(torch.bfloat16)
        for bi, (bm, br) in enumerate(zip(lm, lr)):
            om = bm(inp)
            orf = br(cur_ref)
            print(f"layer{li}.{bi}", cos(om, nhwc(orf)), "stats:",
                  cos(bm.bn1.running_mean, br.bn1.running_mean), cos(bm.bn1.running_var, br.bn1.running_var))
            cur_ref = orf
            inp = nhwc(cur_ref).contiguous().to(torch.bfloat16)
    feat = nhwc(cur_ref).contiguous().to(torch.bfloat16)
    pm = m.avgpool(feat); pr = torch.flatten(r.avgpool(cur_ref), 1)
    print("avgpool", cos(pm, pr))
    print("fc", cos(m.fc(pm), r.fc(pr)))
    print("full", cos(m(x), r(x)))
