"""Training loop (reference train/train.py:18-267), host-side Python.

Same functions, signatures, logging and checkpoint format.  The step body is
the reference's (train.py:112-129): pyramid -> model -> reconstruct -> loss
-> backward -> optimiser step; the compute runs on the umamd HIP kernels and
the optimiser is the fused umamd Adam (identical update rule to
torch.optim.Adam with default betas/eps).
"""
import os
import os.path
from copy import deepcopy
from typing import Optional, Tuple

import torch
from torch.nn import Module
from torch.optim import Optimizer
from torch.utils.data import DataLoader

from umamd import lossfn as LF
from umamd.imageprep import to_device
from umamd.optim import Adam

from . import utils as u
from .utils import Device, Loss, LRAdjuster, ScaleAdjuster

try:
    import tqdm
except ImportError:  # pragma: no cover
    tqdm = None


def save_model(model: Module, save_model_to: str, disc: Optional[Module] = None,
               epoch_number: Optional[int] = None, is_final: bool = False) -> None:
    """state_dict checkpoint as ``final.pt`` / ``epoch_NNN.pt`` (reference :18-48)."""
    os.makedirs(save_model_to, exist_ok=True)
    filename = 'final.pt' if is_final else f'epoch_{epoch_number:03}.pt'
    filepath = os.path.join(save_model_to, filename)
    state_dict = {'model': model.state_dict(), 'disc': disc.state_dict()} \
        if disc is not None else model.state_dict()
    print(f'Saving model to:\n\t{filepath}')
    torch.save(state_dict, filepath)


def _fused_loss(loss_function) -> bool:
    """the umamd fused loss, which fills a deferred recon pyramid itself"""
    from .loss import TukraUncertaintyLoss
    return isinstance(loss_function, TukraUncertaintyLoss)


def train_step(model: Module, left, right, loss_function: Module, optimiser: Optimizer,
               scale: float, scales: int = 4, batch_index: int = 0,
               disc: Optional[Module] = None, disc_clone: Optional[Module] = None,
               disc_optimiser: Optional[Optimizer] = None,
               disc_loss_function: Optional[Module] = None,
               batch_size: Optional[int] = None):
    """One step of the reference loop body (train.py:114-149) without
    logging; returns (disp_loss, error_loss, disc_loss or None) device tensors.
    ``batch_size``: the loader's batch size, which the reference passes to
    run_discriminator (train.py:140-142; on a short last batch every
    prediction is then labelled real); default: this batch's size."""
    images = torch.cat([left, right], dim=1)
    image_pyramid = u.scale_pyramid(images, scales)
    optimiser.zero_grad()
    disparities = model(left, scale)
    if _fused_loss(loss_function):
        with LF.deferred_recon():  # the fused loss forward writes the recon
            recon_pyramid = u.reconstruct_pyramid(disparities, image_pyramid)
    else:  # any other loss reads a recon pyramid computed up front
        recon_pyramid = u.reconstruct_pyramid(disparities, image_pyramid)
    disp_loss, error_loss = loss_function(image_pyramid, disparities, recon_pyramid,
                                          batch_index, disc_clone)
    (disp_loss + error_loss).backward()
    optimiser.step()
    disc_loss = None
    if disc is not None:
        disc_optimiser.zero_grad()
        disc_loss = u.run_discriminator(image_pyramid, recon_pyramid, disc, disc_loss_function,
                                        batch_size if batch_size is not None else left.shape[0])
        disc_loss.backward()
        disc_optimiser.step()
    return disp_loss, error_loss, disc_loss


class _GraphSteps:
    """The captured training step (train.graph.CapturedTrainStep) behind the
    reference loop: one capture per (disparity scale, batch shape), replayed
    for every full batch.  The reference loop's host-side state changes stay
    correct: ``adjust_disparity`` moving the scale recaptures (the old graphs
    are released), ``adjust_learning_rate`` reaches the graph through the
    optimiser's device-side learning rate (umamd.optim.Adam.sync_lr), and a
    batch of another shape (a ragged last batch) takes one eager step.

    Used when the model's parameters are on a HIP device, the optimiser is
    umamd.optim.Adam, the loss is the fused umamd loss and there is no
    discriminator (the adversarial step stays eager).  A DistributedDataParallel
    model must have been built by train.parallel.data_parallel (which builds it
    under the capture stream, see there); a DDP built elsewhere steps eagerly.
    UMAMD_TRAIN_GRAPH=0 turns it off."""

    def __init__(self, model, loss_function, optimiser, scales):
        self.model, self.loss_function, self.optimiser = model, loss_function, optimiser
        self.scales = scales
        self.key = None
        self.cap = None
        self._stream = None

    @property
    def stream(self):
        """ONE stream for every capture and every eager fallback step of the
        loop: autograd's AccumulateGrad nodes remember the stream they were
        created on, and a capture whose backward meets a node of another
        stream (e.g. one an eager ragged-batch step left alive) synchronises
        with it and breaks (measured: segfault in hipStreamEndCapture on the
        recapture after a ragged eager step on the null stream)."""
        if self._stream is None:
            self._stream = getattr(self.model, '_umamd_stream', None) or torch.cuda.Stream()
        return self._stream

    @staticmethod
    def usable(model, loss_function, optimiser, disc) -> bool:
        from torch.nn.parallel import DistributedDataParallel
        if os.environ.get('UMAMD_TRAIN_GRAPH', '1') == '0' or disc is not None:
            return False
        if not hasattr(optimiser, 'sync_lr') or not _fused_loss(loss_function):
            return False
        p = next(model.parameters(), None)
        if p is None or not p.is_cuda:
            return False
        if isinstance(model, DistributedDataParallel):
            from torch import distributed as dist
            if getattr(model, '_umamd_stream', None) is None or \
                    dist.get_backend(model.process_group) != 'nccl':
                return False  # a gloo all-reduce cannot be captured
        return True

    def __call__(self, left, right, scale):
        from .graph import CapturedTrainStep
        key = (float(scale), tuple(left.shape), tuple(right.shape), left.dtype)
        if self.cap is not None and self.key != key and self.key[1:] != key[1:]:
            return None  # another batch shape: the caller steps eagerly
        self.optimiser.sync_lr()
        if self.key != key:
            if self.cap is not None:  # scale changed: drop the old graphs before capturing
                self.cap.close()
            self.cap = None
            torch.cuda.synchronize()
            self.cap = CapturedTrainStep(self.model, self.loss_function, self.optimiser, left,
                                         right, scale, scales=self.scales, stream=self.stream)
            self.key = key
        return self.cap(left, right)


def train_one_epoch(model: Module, loader: DataLoader, loss_function: Module,
                    model_optimiser: Optimizer, scale: float,
                    disc: Optional[Module] = None,
                    disc_optimiser: Optional[Optimizer] = None,
                    disc_loss_function: Optional[Module] = None,
                    epoch_number: Optional[int] = None, scales: int = 4,
                    perceptual_update_freq: int = 10, device: Device = 'cpu',
                    no_pbar: bool = False, rank: int = 0,
                    graph_steps: Optional[_GraphSteps] = None) -> Tuple[float, float]:
    """Reference train/train.py:51-170.  ``graph_steps`` (train_model passes
    one): replay the captured step for full batches (see _GraphSteps)."""
    model.train()
    if disc is not None:
        disc.train()
    running_disp_loss = running_error_loss = running_disc_loss = 0.0
    disp_loss_per_image = unc_loss_per_image = disc_loss_per_image = None
    batch_size = loader.batch_size if loader.batch_size is not None else len(loader)
    description = f'Epoch #{epoch_number}' if epoch_number is not None else 'Epoch'
    disc_clone = deepcopy(disc) if disc is not None else None
    graphs = None
    if graph_steps is not None and _GraphSteps.usable(model, loss_function, model_optimiser,
                                                      disc):
        graphs = graph_steps
    it = tqdm.tqdm(loader, description, unit='batch', disable=(no_pbar or rank > 0)) \
        if tqdm is not None else loader
    for i, image_pair in enumerate(it):
        # a DeviceAugment batch (uint8 + draws) is resized / augmented on the GPU
        left, right = to_device(image_pair, device)
        out = graphs(left, right, scale) if graphs is not None else None
        if out is not None:
            disp_loss, error_loss = out
            disc_loss = None
        elif graphs is not None:
            # a batch of another shape: one eager step on the loop's capture
            # stream (see _GraphSteps.stream)
            cur = torch.cuda.current_stream()
            graphs.stream.wait_stream(cur)
            with torch.cuda.stream(graphs.stream):
                disp_loss, error_loss, disc_loss = train_step(
                    model, left, right, loss_function, model_optimiser, scale, scales, i, disc,
                    disc_clone, disc_optimiser, disc_loss_function, batch_size=batch_size)
            cur.wait_stream(graphs.stream)
        else:
            disp_loss, error_loss, disc_loss = train_step(
                model, left, right, loss_function, model_optimiser, scale, scales, i, disc,
                disc_clone, disc_optimiser, disc_loss_function, batch_size=batch_size)
        if rank == 0:
            running_disp_loss += disp_loss.item()
            running_error_loss += error_loss.item()
            disp_loss_per_image = running_disp_loss / ((i + 1) * batch_size)
            unc_loss_per_image = running_error_loss / ((i + 1) * batch_size)
            if disc_loss is not None:
                running_disc_loss += disc_loss.item()
                disc_loss_per_image = running_disc_loss / ((i + 1) * batch_size)
        if disc is not None and i % perceptual_update_freq == 0:
            disc_clone.load_state_dict(disc.state_dict())
        if rank == 0 and tqdm is not None and hasattr(it, 'set_postfix'):
            it.set_postfix(disp=disp_loss_per_image, unc=unc_loss_per_image,
                           disc=disc_loss_per_image, scale=scale)
    if no_pbar and rank == 0:
        disc_loss_string = f'{disc_loss_per_image:.2e}' \
            if disc_loss_per_image is not None else None
        print(f'{description}:'
              f'\n\tdisparity loss: {disp_loss_per_image:.2e}'
              f'\n\tuncertainty loss: {unc_loss_per_image:.2e}'
              f'\n\tdiscriminator loss: {disc_loss_string}'
              f'\n\tdisparity scale: {scale:.2f}')
    return disp_loss_per_image, unc_loss_per_image, disc_loss_per_image


def train_model(model: Module, loader: DataLoader, loss_function: Module,
                epochs: int, learning_rate: float,
                disc: Optional[Module] = None,
                disc_loss_function: Optional[Module] = None,
                adjust_learning_rate: LRAdjuster = u.adjust_learning_rate,
                adjust_disparity: ScaleAdjuster = u.adjust_disparity,
                perceptual_update_freq: int = 10,
                val_loader: Optional[DataLoader] = None,
                evaluate_every: Optional[int] = None,
                save_evaluation_to: Optional[str] = None,
                save_every: Optional[int] = None,
                save_model_to: Optional[str] = None,
                finetune: bool = False, device: Device = 'cpu',
                no_pbar: bool = False, rank: int = 0) -> Tuple[Loss, Loss]:
    """Epoch loop with the reference's LR / disparity-scale schedules (:173-267)."""
    from .evaluate import evaluate_model
    model_optimiser = Adam(model.parameters(), learning_rate)
    disc_optimiser = Adam(disc.parameters(), learning_rate) if disc is not None else None
    training_losses, validation_metrics = [], []
    graph_steps = _GraphSteps(model, loss_function, model_optimiser, 4)
    for i in range(epochs):
        adjust_learning_rate(model_optimiser, i, learning_rate)
        scale = 1 if finetune else adjust_disparity(i)
        loss = train_one_epoch(model, loader, loss_function, model_optimiser, scale, disc,
                               disc_optimiser, disc_loss_function, epoch_number=(i + 1),
                               perceptual_update_freq=perceptual_update_freq, device=device,
                               no_pbar=no_pbar, rank=rank, graph_steps=graph_steps)
        if rank == 0:
            training_losses.append(loss)
        if evaluate_every is not None and (i + 1) % evaluate_every == 0:
            metrics = evaluate_model(model, val_loader, save_evaluation_to,
                                     epoch_number=(i + 1), is_final=False, scale=scale,
                                     no_pbar=no_pbar, device=device, rank=rank)
            if rank == 0:
                validation_metrics.append(metrics)
        if save_every is not None and (i + 1) % save_every == 0 and rank == 0:
            save_model(model, save_model_to, disc, epoch_number=(i + 1))
    if rank == 0:
        print('Training completed.')
    if save_model_to is not None and rank == 0:
        save_model(model, save_model_to, is_final=True)
    return training_losses, validation_metrics
