"""Evaluation (reference train/evaluate.py:66-196): SURVEY 8(f) "next" row 3
(AUSE/AURG sparsification + 11x11 SSIM); not on the training hot path and not
implemented on the HIP path yet."""


def evaluate_model(*args, **kwargs):
    raise NotImplementedError('umamd: evaluate_model (reference train/evaluate.py) is not '
                              'implemented yet; pass evaluate_every=None to train_model')
