"""Data transforms (reference train/transforms.py): out of scope (SURVEY 2,
CPU data augmentation); the benchmark uses synthetic device-resident pairs.
The names exist so the reference entry points import; using them raises."""


class _Missing:
    def __init__(self, *args, **kwargs):
        raise NotImplementedError(f'umamd: train.transforms.{type(self).__name__} is not '
                                  f'implemented (data pipeline is out of scope)')


class ResizeImage(_Missing):
    pass


class RandomFlip(_Missing):
    pass


class ToTensor(_Missing):
    pass


class RandomAugment(_Missing):
    pass
