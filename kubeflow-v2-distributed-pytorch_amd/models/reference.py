"""Plain-PyTorch reference definitions of the model zoo.

These modules use only ``torch.nn`` layers and exist for two purposes:

1. numerics oracles: tests compare mipipe's fused HIP-kernel models against them
   parameter-for-parameter (same ``state_dict`` keys), and
2. the *stock PyTorch-ROCm comparator* that BASELINE.md asks for (torch DDP +
   MIOpen/hipBLASLt + RCCL on the same MI355X, same model/batch/dtype).

The layer structure and ``state_dict`` key names follow torchvision's ResNet, which
the reference instantiates through ``models.__dict__[arch]()`` (task.py:50-52,
task.py:166-171).  torchvision is not installed in this image, so the layouts are
written from the published architecture (He et al. 2015, ResNet v1.5 with the
stride on the 3x3 conv).
"""
from __future__ import annotations

from typing import List, Optional, Type, Union

import torch
import torch.nn as nn


def conv3x3(cin: int, cout: int, stride: int = 1) -> nn.Conv2d:
    return nn.Conv2d(cin, cout, 3, stride=stride, padding=1, bias=False)


def conv1x1(cin: int, cout: int, stride: int = 1) -> nn.Conv2d:
    return nn.Conv2d(cin, cout, 1, stride=stride, bias=False)


class RefBasicBlock(nn.Module):
    expansion = 1

    def __init__(self, inplanes: int, planes: int, stride: int = 1,
                 downsample: Optional[nn.Module] = None, groups: int = 1, base_width: int = 64):
        super().__init__()
        self.conv1 = conv3x3(inplanes, planes, stride)
        self.bn1 = nn.BatchNorm2d(planes)
        self.relu = nn.ReLU(inplace=True)
        self.conv2 = conv3x3(planes, planes)
        self.bn2 = nn.BatchNorm2d(planes)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x):
        identity = x
        out = self.relu(self.bn1(self.conv1(x)))
        out = self.bn2(self.conv2(out))
        if self.downsample is not None:
            identity = self.downsample(x)
        return self.relu(out + identity)


class RefBottleneck(nn.Module):
    expansion = 4

    def __init__(self, inplanes: int, planes: int, stride: int = 1,
                 downsample: Optional[nn.Module] = None, groups: int = 1, base_width: int = 64):
        super().__init__()
        width = int(planes * (base_width / 64.0)) * groups  # ResNeXt / wide-ResNet width
        self.conv1 = conv1x1(inplanes, width)
        self.bn1 = nn.BatchNorm2d(width)
        self.conv2 = nn.Conv2d(width, width, 3, stride=stride, padding=1, groups=groups,
                               bias=False)
        self.bn2 = nn.BatchNorm2d(width)
        self.conv3 = conv1x1(width, planes * 4)
        self.bn3 = nn.BatchNorm2d(planes * 4)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x):
        identity = x
        out = self.relu(self.bn1(self.conv1(x)))
        out = self.relu(self.bn2(self.conv2(out)))
        out = self.bn3(self.conv3(out))
        if self.downsample is not None:
            identity = self.downsample(x)
        return self.relu(out + identity)


class RefResNet(nn.Module):
    def __init__(self, block: Type[Union[RefBasicBlock, RefBottleneck]], layers: List[int],
                 num_classes: int = 1000, in_chans: int = 3, groups: int = 1,
                 width_per_group: int = 64):
        super().__init__()
        self.inplanes = 64
        self.groups, self.base_width = groups, width_per_group
        self.conv1 = nn.Conv2d(in_chans, 64, 7, stride=2, padding=3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(3, stride=2, padding=1)
        self.layer1 = self._make_layer(block, 64, layers[0])
        self.layer2 = self._make_layer(block, 128, layers[1], stride=2)
        self.layer3 = self._make_layer(block, 256, layers[2], stride=2)
        self.layer4 = self._make_layer(block, 512, layers[3], stride=2)
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))
        self.fc = nn.Linear(512 * block.expansion, num_classes)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.ones_(m.weight)
                nn.init.zeros_(m.bias)

    def _make_layer(self, block, planes, blocks, stride=1):
        downsample = None
        if stride != 1 or self.inplanes != planes * block.expansion:
            downsample = nn.Sequential(conv1x1(self.inplanes, planes * block.expansion, stride),
                                       nn.BatchNorm2d(planes * block.expansion))
        layers = [block(self.inplanes, planes, stride, downsample, self.groups, self.base_width)]
        self.inplanes = planes * block.expansion
        for _ in range(1, blocks):
            layers.append(block(self.inplanes, planes, groups=self.groups,
                                base_width=self.base_width))
        return nn.Sequential(*layers)

    def forward(self, x):
        x = self.maxpool(self.relu(self.bn1(self.conv1(x))))
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        x = torch.flatten(self.avgpool(x), 1)
        return self.fc(x)


_RESNET_CFG = {  # arch: (block, layers, groups, width_per_group)
    "resnet18": (RefBasicBlock, [2, 2, 2, 2], 1, 64),
    "resnet34": (RefBasicBlock, [3, 4, 6, 3], 1, 64),
    "resnet50": (RefBottleneck, [3, 4, 6, 3], 1, 64),
    "resnet101": (RefBottleneck, [3, 4, 23, 3], 1, 64),
    "resnet152": (RefBottleneck, [3, 8, 36, 3], 1, 64),
    "wide_resnet50_2": (RefBottleneck, [3, 4, 6, 3], 1, 128),
    "wide_resnet101_2": (RefBottleneck, [3, 4, 23, 3], 1, 128),
    "resnext50_32x4d": (RefBottleneck, [3, 4, 6, 3], 32, 4),
    "resnext101_32x8d": (RefBottleneck, [3, 4, 23, 3], 32, 8),
}


def ref_resnet(arch: str, num_classes: int = 1000, in_chans: int = 3) -> RefResNet:
    block, layers, groups, width = _RESNET_CFG[arch]
    return RefResNet(block, layers, num_classes=num_classes, in_chans=in_chans, groups=groups,
                     width_per_group=width)


class RefMnistCNN(nn.Module):
    """Small CNN for the MNIST-shape correctness config (BASELINE config 1)."""

    def __init__(self, num_classes: int = 10, in_chans: int = 1):
        super().__init__()
        self.conv1 = nn.Conv2d(in_chans, 32, 3, padding=1, bias=False)
        self.bn1 = nn.BatchNorm2d(32)
        self.conv2 = nn.Conv2d(32, 64, 3, stride=2, padding=1, bias=False)
        self.bn2 = nn.BatchNorm2d(64)
        self.conv3 = nn.Conv2d(64, 128, 3, stride=2, padding=1, bias=False)
        self.bn3 = nn.BatchNorm2d(128)
        self.fc1 = nn.Linear(128, 128)
        self.fc2 = nn.Linear(128, num_classes)

    def forward(self, x):
        x = torch.relu(self.bn1(self.conv1(x)))
        x = torch.relu(self.bn2(self.conv2(x)))
        x = torch.relu(self.bn3(self.conv3(x)))
        x = x.mean(dim=(2, 3))
        return self.fc2(torch.relu(self.fc1(x)))


# ----------------------------------------------------------------------------- BERT (stock)
class _RefBertLayer(nn.Module):
    def __init__(self, H: int, heads: int, inter: int, eps: float, p: float, pa: float):
        super().__init__()
        self.heads, self.pa = heads, pa
        self.attention = nn.Module()
        self.attention.self = nn.Module()
        self.attention.self.query = nn.Linear(H, H)
        self.attention.self.key = nn.Linear(H, H)
        self.attention.self.value = nn.Linear(H, H)
        self.attention.output = nn.Module()
        self.attention.output.dense = nn.Linear(H, H)
        self.attention.output.LayerNorm = nn.LayerNorm(H, eps=eps)
        self.intermediate = nn.Module()
        self.intermediate.dense = nn.Linear(H, inter)
        self.output = nn.Module()
        self.output.dense = nn.Linear(inter, H)
        self.output.LayerNorm = nn.LayerNorm(H, eps=eps)
        self.drop = nn.Dropout(p)

    def forward(self, h, mask):
        B, S, H = h.shape
        sa = self.attention.self

        def split(t):
            return t.view(B, S, self.heads, H // self.heads).transpose(1, 2)

        q, k, v = split(sa.query(h)), split(sa.key(h)), split(sa.value(h))
        ctx = torch.nn.functional.scaled_dot_product_attention(
            q, k, v, attn_mask=mask, dropout_p=self.pa if self.training else 0.0)
        ctx = ctx.transpose(1, 2).reshape(B, S, H)
        a = self.drop(self.attention.output.dense(ctx))
        h1 = self.attention.output.LayerNorm(a + h)
        f = torch.nn.functional.gelu(self.intermediate.dense(h1))
        f2 = self.drop(self.output.dense(f))
        return self.output.LayerNorm(f2 + h1)


class RefBertForMaskedLM(nn.Module):
    """HuggingFace-``BertForMaskedLM``-keyed stock PyTorch BERT (torch.nn + SDPA): oracle for
    :class:`mipipe.models.bert.BertForMaskedLM` and the BERT stock comparator."""

    def __init__(self, vocab_size=30522, hidden_size=768, num_hidden_layers=12,
                 num_attention_heads=12, intermediate_size=3072, max_position_embeddings=512,
                 type_vocab_size=2, layer_norm_eps=1e-12, hidden_dropout_prob=0.1,
                 attention_probs_dropout_prob=0.1):
        super().__init__()
        H = hidden_size
        self.bert = nn.Module()
        e = self.bert.embeddings = nn.Module()
        e.word_embeddings = nn.Embedding(vocab_size, H)
        e.position_embeddings = nn.Embedding(max_position_embeddings, H)
        e.token_type_embeddings = nn.Embedding(type_vocab_size, H)
        e.LayerNorm = nn.LayerNorm(H, eps=layer_norm_eps)
        self.bert.encoder = nn.Module()
        self.bert.encoder.layer = nn.ModuleList(
            [_RefBertLayer(H, num_attention_heads, intermediate_size, layer_norm_eps,
                           hidden_dropout_prob, attention_probs_dropout_prob)
             for _ in range(num_hidden_layers)])
        self.cls = nn.Module()
        pr = self.cls.predictions = nn.Module()
        pr.transform = nn.Module()
        pr.transform.dense = nn.Linear(H, H)
        pr.transform.LayerNorm = nn.LayerNorm(H, eps=layer_norm_eps)
        pr.bias = nn.Parameter(torch.zeros(vocab_size))
        pr.decoder = nn.Linear(H, vocab_size)
        pr.decoder.weight = e.word_embeddings.weight
        pr.decoder.bias = pr.bias
        self.drop = nn.Dropout(hidden_dropout_prob)
        for mod in self.modules():  # HF BertPreTrainedModel._init_weights (std 0.02)
            if isinstance(mod, nn.Linear):
                nn.init.normal_(mod.weight, 0.0, 0.02)
                if mod.bias is not None:
                    nn.init.zeros_(mod.bias)
            elif isinstance(mod, nn.Embedding):
                nn.init.normal_(mod.weight, 0.0, 0.02)

    def forward(self, input_ids, attention_mask=None, token_type_ids=None, masked_positions=None):
        B, S = input_ids.shape
        e = self.bert.embeddings
        pos = torch.arange(S, device=input_ids.device)[None, :]
        tt = torch.zeros_like(input_ids) if token_type_ids is None else token_type_ids
        h = e.word_embeddings(input_ids) + e.position_embeddings(pos) + e.token_type_embeddings(tt)
        h = self.drop(e.LayerNorm(h))
        mask = None
        if attention_mask is not None:
            mask = ((1.0 - attention_mask.to(h.dtype)) * -10000.0)[:, None, None, :]
        for layer in self.bert.encoder.layer:
            h = layer(h, mask)
        h = h.reshape(B * S, -1)
        if masked_positions is not None:
            rows = (masked_positions + torch.arange(B, device=h.device)[:, None] * S).reshape(-1)
            h = h.index_select(0, rows)
        pr = self.cls.predictions
        t = pr.transform.LayerNorm(torch.nn.functional.gelu(pr.transform.dense(h)))
        return pr.decoder(t)

    def loss(self, logits, labels):
        lf = logits if logits.dtype == torch.float64 else logits.float()
        return torch.nn.functional.cross_entropy(lf, labels.reshape(-1), ignore_index=-100)


def ref_bert(arch: str = "bert_base", **kw) -> RefBertForMaskedLM:
    if arch == "bert_tiny":
        kw = {**dict(hidden_size=128, num_hidden_layers=2, num_attention_heads=2,
                     intermediate_size=512), **kw}
    return RefBertForMaskedLM(**kw)


# ----------------------------------------------------------------------------- VGG / AlexNet
_VGG_CFGS = {
    "vgg11": [64, "M", 128, "M", 256, 256, "M", 512, 512, "M", 512, 512, "M"],
    "vgg13": [64, 64, "M", 128, 128, "M", 256, 256, "M", 512, 512, "M", 512, 512, "M"],
    "vgg16": [64, 64, "M", 128, 128, "M", 256, 256, 256, "M", 512, 512, 512, "M",
              512, 512, 512, "M"],
    "vgg19": [64, 64, "M", 128, 128, "M", 256, 256, 256, 256, "M", 512, 512, 512, 512, "M",
              512, 512, 512, 512, "M"],
}


class RefVGG(nn.Module):
    """torchvision-structured VGG (plain torch.nn) — oracle / stock comparator."""

    def __init__(self, arch: str = "vgg16", num_classes: int = 1000, dropout: float = 0.5):
        super().__init__()
        bn = arch.endswith("_bn")
        layers: List[nn.Module] = []
        c = 3
        for v in _VGG_CFGS[arch.replace("_bn", "")]:
            if v == "M":
                layers.append(nn.MaxPool2d(2, 2))
                continue
            layers.append(nn.Conv2d(c, v, 3, padding=1))
            if bn:
                layers.append(nn.BatchNorm2d(v))
            layers.append(nn.ReLU(inplace=True))
            c = v
        self.features = nn.Sequential(*layers)
        self.avgpool = nn.AdaptiveAvgPool2d((7, 7))
        self.classifier = nn.Sequential(
            nn.Linear(512 * 7 * 7, 4096), nn.ReLU(True), nn.Dropout(dropout),
            nn.Linear(4096, 4096), nn.ReLU(True), nn.Dropout(dropout),
            nn.Linear(4096, num_classes))

    def forward(self, x):
        x = self.avgpool(self.features(x))
        return self.classifier(torch.flatten(x, 1))


class RefAlexNet(nn.Module):
    def __init__(self, num_classes: int = 1000, dropout: float = 0.5):
        super().__init__()
        self.features = nn.Sequential(
            nn.Conv2d(3, 64, 11, stride=4, padding=2), nn.ReLU(True), nn.MaxPool2d(3, 2),
            nn.Conv2d(64, 192, 5, padding=2), nn.ReLU(True), nn.MaxPool2d(3, 2),
            nn.Conv2d(192, 384, 3, padding=1), nn.ReLU(True),
            nn.Conv2d(384, 256, 3, padding=1), nn.ReLU(True),
            nn.Conv2d(256, 256, 3, padding=1), nn.ReLU(True), nn.MaxPool2d(3, 2))
        self.avgpool = nn.AdaptiveAvgPool2d((6, 6))
        self.classifier = nn.Sequential(
            nn.Dropout(dropout), nn.Linear(256 * 6 * 6, 4096), nn.ReLU(True),
            nn.Dropout(dropout), nn.Linear(4096, 4096), nn.ReLU(True),
            nn.Linear(4096, num_classes))

    def forward(self, x):
        x = self.avgpool(self.features(x))
        return self.classifier(torch.flatten(x, 1))
