"""Drop-in for the reference's communicator.py (see the package's communicator module)."""
from _mx_pkg import PKG

Communicator = PKG.Communicator
decenCommunicator = PKG.decenCommunicator
ChocoCommunicator = PKG.ChocoCommunicator
centralizedCommunicator = PKG.centralizedCommunicator
