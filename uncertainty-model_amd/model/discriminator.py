"""RandomDiscriminator (reference model/discriminator.py:13-86).

Adversarial training (BASELINE config 3) is the first "next" row of SURVEY
8(f) and is not implemented on the HIP path yet.  The class exists so the
reference entry points import unchanged; constructing it raises.
"""
import torch.nn as nn


class RandomDiscriminator(nn.Module):
    def __init__(self, *args, **kwargs) -> None:
        super().__init__()
        raise NotImplementedError('umamd: the adversarial path (RandomDiscriminator, '
                                  'reference model/discriminator.py) is not implemented yet')
