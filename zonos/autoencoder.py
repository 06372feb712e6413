"""`zonos.autoencoder` import surface (reference zonos/autoencoder.py): DACAutoencoder on the HIP
DAC decoder / encoder (zonos_amd/autoencoder.py)."""
from zonos_amd.autoencoder import DACAutoencoder  # noqa: F401
