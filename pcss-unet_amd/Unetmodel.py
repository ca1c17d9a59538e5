"""Drop-in replacement for the reference module `Unetmodel`
(/root/reference/Unetmodel.py): `from Unetmodel import Unet, DoubleConv`
now resolves to the MI355X-native implementation (nsm_amd)."""
import os

from nsm_amd.unet import DoubleConv, Unet  # noqa: F401


def makefilepath(folder_path):
    """Unetmodel.py:152-154"""
    if not os.path.exists(folder_path):
        os.makedirs(folder_path)
