"""pgmorl_amd -- MI355X-native (gfx950) PG-MORL MOPG hot path.

Hand-written HIP kernels in ``csrc/`` behind the C ABI ``include/pgm_abi.h`` (libpgm.so),
a device-resident task runtime (``runtime.TaskBatch``) and the reference-compatible host
API (Sample / Task / EP / OptGraph / MOPG population drop-in).
"""
__version__ = '0.1.0'
