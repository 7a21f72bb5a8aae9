"""CPU: the MLP's split-K weight-gradient Linear matches plain autograd."""
import torch

from avr_amd import model as M


def test_split_k_linear_matches_autograd():
    torch.manual_seed(0)
    for n in (100, M._WGRAD_ROWS * 3 + 17):
        x = torch.randn(n, 48, requires_grad=True)
        w = torch.randn(32, 48, requires_grad=True)
        gy = torch.randn(n, 32)
        y = M._Linear.apply(x, w, torch.float32)
        y.backward(gy)
        x2 = x.detach().clone().requires_grad_(True)
        w2 = w.detach().clone().requires_grad_(True)
        (x2 @ w2.t()).backward(gy)
        torch.testing.assert_close(y, x2 @ w2.t())
        torch.testing.assert_close(x.grad, x2.grad)
        torch.testing.assert_close(w.grad, w2.grad, rtol=1e-4, atol=1e-4)
        assert w.grad.dtype == torch.float32


def test_mlp_shapes_and_relu_chain():
    cfg = dict(n_neurons=16, n_hidden_layers=2, activation="ReLU")
    mlp = M.MLP(5, 7, cfg)
    x = torch.randn(9, 5)
    ref = x
    for i, lin in enumerate(mlp.layers):
        ref = ref @ lin.weight.t()
        if i + 1 < len(mlp.layers):
            ref = torch.relu(ref)
    torch.testing.assert_close(mlp(x), ref)
