"""Training schedules (learning rate, scheduled sampling, MIXER, SCB).

Formulas reproduce the reference:
  * LR step decay               -- ``/root/reference/utils.py:22-28``
  * scheduled-sampling prob      -- ``/root/reference/train.py:109-114``
  * MIXER annealing              -- ``/root/reference/train.py:136-140``
  * SCB (consensus) annealing    -- ``/root/reference/train.py:158-162``
"""
import math


def lr_at(opt, epoch):
    """``lr0 * 0.1 ** (epoch // lr_update)``."""
    return opt.learning_rate * (0.1 ** (epoch // opt.lr_update))


def adjust_learning_rate(opt, optimizer, epoch):
    lr = lr_at(opt, epoch)
    for group in optimizer.param_groups:
        group['lr'] = lr
    return lr


def ss_prob(opt, epoch):
    """Probability of feeding a model sample instead of the GT token."""
    if not (opt.use_ss == 1 and epoch >= opt.use_ss_after):
        return 0.0
    annealing = opt.ss_k / (opt.ss_k + math.exp((epoch - opt.use_ss_after) / opt.ss_k))
    return min(1.0 - annealing, opt.ss_max_prob)


def mixer_from(opt, epoch, seq_length):
    """First time step that is sampled (MIXER); ``opt.mixer_from`` unless -1."""
    if opt.mixer_from != -1:
        return opt.mixer_from
    annealed = seq_length - int(math.ceil((epoch - opt.use_rl_after + 1) /
                                          opt.mixer_descrease_every))
    return max(1, annealed)


def scb_captions(opt, epoch, seq_per_img):
    """Number of lowest scores averaged into the consensus baseline."""
    if opt.scb_captions != -1:
        return opt.scb_captions
    annealed = int(math.ceil((epoch - opt.use_cst_after + 1) / opt.cst_increase_every))
    return min(annealed, seq_per_img - 1)
