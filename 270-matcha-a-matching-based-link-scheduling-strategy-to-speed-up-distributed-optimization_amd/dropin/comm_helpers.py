"""Drop-in for the reference's comm_helpers.py."""
from _mx_pkg import PKG

flatten_tensors = PKG.flatten_tensors
unflatten_tensors = PKG.unflatten_tensors
communicate = PKG.comm_helpers.communicate
