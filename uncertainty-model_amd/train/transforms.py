"""Dict-wise stereo transforms (reference train/transforms.py:15-129).

These run in DataLoader worker processes on the host (PIL / numpy / torch
CPU), exactly where the reference runs them; they never touch the HIP
library (one process per GPU owns it).  torchvision is not a dependency:
the three torchvision ops the reference wraps are restated with their
torchvision semantics --

  * ``Resize(size)``          PIL ``Image.resize((w, h), BILINEAR)`` for PIL
                              images (torchvision's PIL path); bilinear with
                              antialias for tensors (align_corners=False)
  * ``ToTensor()``            HWC uint8 -> CHW float in [0, 1]
  * ``RandomHorizontalFlip(1)``  mirror along the width

Randomness uses ``numpy.random`` as the reference does (:56, :120-124), so a
seeded worker reproduces the reference's flip/augment decisions.
"""
from typing import Dict, Tuple

import numpy as np
from numpy import random

import torch
import torch.nn.functional as F
from torch import Tensor

try:
    from PIL import Image
except ImportError:  # pragma: no cover - PIL ships with the image
    Image = None

ImageDict = Dict[str, Tensor]
BoundsTuple = Tuple[float, float]
ImageSize = Tuple[int, int]


def _is_pil(x) -> bool:
    return Image is not None and isinstance(x, Image.Image)


def resize(x, size: ImageSize):
    """torchvision.transforms.functional.resize with a (h, w) size and the
    default bilinear interpolation."""
    h, w = int(size[0]), int(size[1])
    if _is_pil(x):
        return x.resize((w, h), Image.BILINEAR)
    if not isinstance(x, Tensor):
        raise TypeError(f'resize: PIL image or tensor expected, got {type(x)}')
    squeeze = x.dim() == 3
    t = x.unsqueeze(0) if squeeze else x
    dt = t.dtype
    out = F.interpolate(t.float(), size=(h, w), mode='bilinear', align_corners=False,
                        antialias=True)
    if dt == torch.uint8:
        out = out.round().clamp(0, 255).to(dt)
    else:
        out = out.to(dt)
    return out.squeeze(0) if squeeze else out


def to_tensor(pic) -> Tensor:
    """torchvision.transforms.functional.to_tensor for PIL images and HWC
    numpy arrays (8-bit -> /255)."""
    if isinstance(pic, np.ndarray):
        arr = pic if pic.ndim == 3 else pic[:, :, None]
        t = torch.from_numpy(np.ascontiguousarray(arr)).permute(2, 0, 1).contiguous()
        return t.float().div(255) if t.dtype == torch.uint8 else t
    if not _is_pil(pic):
        raise TypeError(f'to_tensor: PIL image or ndarray expected, got {type(pic)}')
    if pic.mode == 'I':
        arr = np.array(pic, np.int32, copy=True)
    elif pic.mode == 'I;16':
        arr = np.array(pic, np.int16, copy=True)
    elif pic.mode == 'F':
        arr = np.array(pic, np.float32, copy=True)
    elif pic.mode == '1':
        arr = 255 * np.array(pic, np.uint8, copy=True)
    else:
        arr = np.array(pic, np.uint8, copy=True)
    t = torch.from_numpy(arr)
    t = t.view(pic.size[1], pic.size[0], len(pic.getbands())).permute(2, 0, 1).contiguous()
    return t.float().div(255) if t.dtype == torch.uint8 else t


def hflip(x):
    if _is_pil(x):
        return x.transpose(Image.FLIP_LEFT_RIGHT)
    return x.flip(-1)


class ResizeImage:
    """Resize the stereo images grouped in a dictionary (reference :15-29)."""

    def __init__(self, size: ImageSize = (256, 512)) -> None:
        self.size = size

    def transform(self, x):
        return resize(x, self.size)

    def __call__(self, image_pair: ImageDict) -> ImageDict:
        return {'left': self.transform(image_pair['left']),
                'right': self.transform(image_pair['right'])}


class ToTensor:
    """Convert stereo PIL images grouped in a dictionary (reference :32-41)."""

    def transform(self, x):
        return to_tensor(x)

    def __call__(self, image_pair: ImageDict) -> ImageDict:
        return {'left': self.transform(image_pair['left']),
                'right': self.transform(image_pair['right'])}


class RandomFlip:
    """Random horizontal flip of both views (reference :44-60; like the
    reference it does not swap left and right)."""

    def __init__(self, p: float = 0.5) -> None:
        self.probability = p

    def transform(self, x):
        return hflip(x)

    def __call__(self, image_pair: ImageDict) -> ImageDict:
        if random.random() < self.probability:
            image_pair['left'] = self.transform(image_pair['left'])
            image_pair['right'] = self.transform(image_pair['right'])
        return image_pair


class RandomAugment:
    """Random gamma / brightness / colour shift of both views (reference
    :63-129)."""

    def __init__(self, p: float, gamma: BoundsTuple, brightness: BoundsTuple,
                 colour: BoundsTuple) -> None:
        self.probability = p
        self.gamma = gamma
        self.brightness = brightness
        self.colour = colour

    def shift_gamma(self, x: Tensor, gamma: float) -> Tensor:
        return x ** gamma

    def shift_brightness(self, x: Tensor, brightness: float) -> Tensor:
        return x * brightness

    def shift_colour(self, x: Tensor, colour: Tensor) -> Tensor:
        return x * colour.unsqueeze(-1).unsqueeze(-1)

    def transform(self, x: Tensor, gamma: float, brightness: float, colour: Tensor) -> Tensor:
        x = self.shift_gamma(x, gamma)
        x = self.shift_brightness(x, brightness)
        x = self.shift_colour(x, colour)
        return torch.clamp(x, 0, 1)

    def __call__(self, image_pair: ImageDict) -> ImageDict:
        left, right = image_pair['left'], image_pair['right']
        if random.random() < self.probability:
            g = random.uniform(*self.gamma)
            b = random.uniform(*self.brightness)
            c = torch.tensor(random.uniform(*self.colour, 3), dtype=torch.float)
            left = self.transform(left, g, b, c)
            right = self.transform(right, g, b, c)
        return {'left': left, 'right': right}


class Compose:
    """torchvision.transforms.Compose (the reference's main.py builds its
    pipelines with it; provided here for images without torchvision)."""

    def __init__(self, transforms) -> None:
        self.transforms = list(transforms)

    def __call__(self, x):
        for t in self.transforms:
            x = t(x)
        return x


class DeviceAugment:
    """The augmenting pipeline with its arithmetic on the GPU (umamd.imageprep):
    a drop-in for ``Compose([ResizeImage(size), RandomFlip(0.5), ToTensor(),
    RandomAugment(0.5, ...)])`` (reference main.py:78-89) whose workers only
    convert the decoded PIL pair to uint8 arrays and draw the flip / augment
    parameters in the reference's numpy order.  The batch then carries
    uint8 images + parameters, and ``train.train`` (or
    ``umamd.imageprep.to_device``) turns it into the f32 [N, 3, H, W] pair on
    the device in two kernel launches.  ``augment=False`` gives the
    no-augment pipeline (ResizeImage + ToTensor, main.py:91-93)."""

    def __init__(self, size: ImageSize = (256, 512), flip_p: float = 0.5,
                 augment_p: float = 0.5, gamma: BoundsTuple = (0.8, 1.2),
                 brightness: BoundsTuple = (0.5, 2.0), colour: BoundsTuple = (0.8, 1.2),
                 augment: bool = True) -> None:
        from umamd.imageprep import StereoDraws
        self.draws = StereoDraws(flip_p, augment_p, gamma, brightness, colour, augment, size)

    def __call__(self, image_pair):
        return self.draws({'left': np.asarray(image_pair['left']),
                           'right': np.asarray(image_pair['right'])})
