"""compressai.layers helpers used by the reference (conv3x3, subpel_conv3x3)
plus ``conv1x1`` (layers/Masked_Attention.py:11-13).  Same module structure, so
the state_dict keys match (e.g. ``h_mean_s.0.0.weight`` for a subpel conv)."""
import torch.nn as nn


def conv3x3(in_ch, out_ch, stride=1):
    return nn.Conv2d(in_ch, out_ch, kernel_size=3, stride=stride, padding=1)


def subpel_conv3x3(in_ch, out_ch, r=1):
    return nn.Sequential(nn.Conv2d(in_ch, out_ch * r ** 2, kernel_size=3, padding=1),
                         nn.PixelShuffle(r))


def conv1x1(in_ch, out_ch, stride=1):
    return nn.Conv2d(in_ch, out_ch, kernel_size=1, stride=stride)


def conv(in_channels, out_channels, kernel_size=5, stride=2):
    """models/AutoEncoderRGB_Journal.py:20-27."""
    return nn.Conv2d(in_channels, out_channels, kernel_size=kernel_size, stride=stride,
                     padding=kernel_size // 2)


def deconv(in_channels, out_channels, kernel_size=5, stride=2):
    """models/AutoEncoderRGB_Journal.py:75-83."""
    return nn.ConvTranspose2d(in_channels, out_channels, kernel_size=kernel_size, stride=stride,
                              output_padding=stride - 1, padding=kernel_size // 2)
