"""Small helpers of the HiFi-GAN code base (hifigan/xutils.py:25-38)."""


def get_padding(kernel_size: int, dilation: int = 1) -> int:
    return int((kernel_size * dilation - dilation) / 2)


def init_weights(m, mean: float = 0.0, std: float = 0.01):
    if "Conv" in m.__class__.__name__:
        m.weight.data.normal_(mean, std)
