"""Drop-in ``hifigan`` package (main.py:136-138): Generator / Denoiser on MI355X HIP kernels."""
