"""Drop-in for the reference's compressors.py."""
from _mx_pkg import PKG

get_top_k = PKG.get_top_k
