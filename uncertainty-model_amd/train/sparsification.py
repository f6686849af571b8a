"""Sparsification curves, AUSE and AURG (reference train/sparsification.py:8-61)
on the HIP path (umamd.evalfn): 11x11 average pooling, a segmented radix
sort per (image, view) and the 100-step curve on the device."""
import torch
from torch import Tensor

from umamd import evalfn as EF

from .utils import Device


def curve(oracle_error: Tensor, predicted_error: Tensor, kernel_size: int = 11,
          steps: int = 100, device: Device = 'cpu') -> Tensor:
    return EF.sparsification_curve(oracle_error, predicted_error, kernel_size, steps).to(device)


def random_curve(oracle_error: Tensor, kernel_size: int = 11, steps: int = 100,
                 device: Device = 'cpu') -> Tensor:
    random_error = torch.rand_like(oracle_error)
    return curve(oracle_error, random_error, kernel_size, steps, device)


def error(oracle_curve: Tensor, predicted_curve: Tensor) -> Tensor:
    return predicted_curve - oracle_curve


def ause(oracle_curve: Tensor, predicted_curve: Tensor) -> Tensor:
    if len(oracle_curve) != len(predicted_curve):
        raise Exception('Oracle and Predicted sparsification curves have different step sizes.')
    return error(oracle_curve, predicted_curve).sum() / len(oracle_curve)


def aurg(predicted_curve: Tensor, random_curve: Tensor) -> Tensor:
    return ause(predicted_curve, random_curve)
