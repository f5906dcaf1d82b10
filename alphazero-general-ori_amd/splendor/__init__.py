"""MI355X-native Splendor engine (HIP, gfx950) behind the reference's Game plug-in API.

Modules:
  _lib          ctypes binding of libsplendor_amd.so (fails loudly if missing)
  env           batched device-resident environment (SplendorEngine, RolloutBatch)
  SplendorGame  the reference's Game interface (SplendorGame.py:11-86), engine-backed
"""
