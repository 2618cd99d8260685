"""BatchNormAct2d (fused BN + residual + ReLU module): CPU semantics = the unfused composition."""
import torch
import torch.nn as nn
import torch.nn.functional as F

from grace_amd.models import resnet18, resnet50, resnet9
from grace_amd.ops.bnact import BatchNormAct2d


def _ref(bn, x, res, relu):
    y = F.batch_norm(x, bn.running_mean, bn.running_var, bn.weight, bn.bias, bn.training, bn.momentum, bn.eps)
    if res is not None:
        y = y + res
    return F.relu(y) if relu else y


def test_bnact_module_matches_composition_cpu():
    torch.manual_seed(0)
    for relu in (False, True):
        for with_res in (False, True):
            m = BatchNormAct2d(16, relu=relu)
            r = nn.BatchNorm2d(16)
            r.load_state_dict(m.state_dict())
            x = torch.randn(4, 16, 5, 5, requires_grad=True)
            res = torch.randn(4, 16, 5, 5, requires_grad=True) if with_res else None
            y = m(x, res)
            y0 = _ref(r, x, res, relu)
            torch.testing.assert_close(y, y0)
            torch.testing.assert_close(m.running_mean, r.running_mean)
            assert int(m.num_batches_tracked) == 1
            m.eval()
            r.eval()
            torch.testing.assert_close(m(x, res), _ref(r, x, res, relu))


def test_bnact_state_dict_keys_are_batchnorm_keys():
    assert set(BatchNormAct2d(8, relu=True).state_dict()) == set(nn.BatchNorm2d(8).state_dict())
    assert isinstance(BatchNormAct2d(8), nn.BatchNorm2d)


def test_model_parameter_counts_unchanged():
    # torchvision's counts: the fused modules keep every parameter
    assert sum(p.numel() for p in resnet50().parameters()) == 25557032
    assert sum(p.numel() for p in resnet18().parameters()) == 11689512
    assert sum(p.numel() for p in resnet9().parameters()) == 6573120
