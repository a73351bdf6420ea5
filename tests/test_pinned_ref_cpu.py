"""The decision-pinned float64 reference (tests/pinned_ref.py) that the fp32 GPU model test
compares against: with its own float64 decisions it must equal the mipipe module tree evaluated
in float64 on the CPU (the same graph, independent code), and feeding those decisions back as a
tape must reproduce the same gradients bit for bit."""
import torch

from pinned_ref import pinned_grads


def test_pinned_reference_matches_module_tree_float64():
    from mipipe.models import create_model
    torch.manual_seed(0)
    m = create_model("resnet18", num_classes=10, compute_dtype=torch.float64).double()
    state = {k: v.clone() for k, v in m.state_dict().items()}
    names = [n for n, _ in m.named_parameters()]
    x = torch.randn(8, 3, 32, 32, dtype=torch.float64)
    y = torch.randint(0, 10, (8,))
    out = m(x)
    loss = torch.nn.functional.cross_entropy(out, y)
    loss.backward()
    logits, loss_r, g, pin = pinned_grads(state, names, x, y, None)
    assert len(pin.own.relu_masks) == 16 and pin.own.pool is not None
    assert torch.allclose(out, logits, rtol=1e-10, atol=1e-12)
    assert abs(loss.item() - loss_r.item()) < 1e-12
    grads = dict(m.named_parameters())
    for n in names:
        a, b = grads[n].grad, g[n]
        assert ((a - b).norm() / b.norm()).item() < 1e-10, n
    # replaying its own decisions is the identity
    _, _, g2, _ = pinned_grads(state, names, x, y, pin.own)
    for n in names:
        assert torch.equal(g[n], g2[n]), n


def test_pinned_reference_follows_a_flipped_decision():
    """Flip one ReLU decision of layer4 and the pinned gradients move, while an unflipped tape
    leaves them unchanged: the reference really routes gradients by the tape."""
    from mipipe.models import create_model
    torch.manual_seed(1)
    m = create_model("resnet18", num_classes=10)
    state = m.state_dict()
    names = [n for n, _ in m.named_parameters()]
    x = torch.randn(8, 3, 32, 32)
    y = torch.randint(0, 10, (8,))
    _, _, g, pin = pinned_grads(state, names, x, y, None)
    tape = pin.own
    tape.relu_masks[-2] = tape.relu_masks[-2].clone()
    tape.relu_masks[-2].view(-1)[3] ^= True
    _, _, g2, _ = pinned_grads(state, names, x, y, tape)
    moved = [n for n in names if not torch.equal(g[n], g2[n])]
    assert "layer4.1.bn1.weight" in moved and "layer1.0.conv1.weight" in moved
