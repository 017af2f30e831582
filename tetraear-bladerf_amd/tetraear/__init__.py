"""tetraear (MI355X build): the demod + lower-MAC hot path of TetraEar-BladeRF on gfx950.

The package keeps the reference's ``tetraear.signal`` / ``tetraear.core`` module surface for the
hot path; numeric work runs in libtetra_hip.so (see include/tetra_hip.h).
"""
__version__ = "0.1.0"
