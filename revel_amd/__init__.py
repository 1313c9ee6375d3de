"""revel_amd -- MI355X-native CRC32C engine for Revel's WAL record path.

Python mirror of the reference's WAL surface (guimingyue/revel @ v0) over the
C-ABI of ``librevel_wal.so`` (include/revel_wal.h):

* :mod:`revel_amd.crc`  -- ``value/extend/mask/unmask``   (src/util/crc.rs)
* :mod:`revel_amd.env`  -- writable / sequential files    (src/env.rs)
* :mod:`revel_amd.log`  -- ``Writer`` / ``Reader``        (src/log_writer.rs, src/log_reader.rs)
* :mod:`revel_amd.gpu`  -- device-resident CRC engine (gfx950 HIP kernels)
"""
from ._lib import (BLOCK_SIZE, FIRST_TYPE, FULL_TYPE, HEADER_SIZE, LAST_TYPE, MIDDLE_TYPE, ZERO_TYPE,
                   RevelError, lib)
from . import crc, env, log, gpu  # noqa: F401

__all__ = ["BLOCK_SIZE", "HEADER_SIZE", "ZERO_TYPE", "FULL_TYPE", "FIRST_TYPE", "MIDDLE_TYPE", "LAST_TYPE",
           "RevelError", "lib", "crc", "env", "log", "gpu"]
