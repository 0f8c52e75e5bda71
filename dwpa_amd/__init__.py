"""dwpa_amd -- MI355X-native m22000 PMK derivation + verification engine (drop-in for dwpa's hot path).

The product is ``lib/libdwpa22000.so`` (HIP kernels for gfx950 behind the C ABI in ``include/dwpa22000.h``);
this package is its Python host side:

* :func:`check_key_m22000` -- PHP-shaped mirror of ``web/common.php:157-307`` (server key check)
* :func:`check_batch`      -- bulk form (put_work / rkg loops)
* :func:`pbkdf2_pmk`       -- PMK derivation
* :class:`Scan`            -- device-resident scan of HBM dictionaries / keyspaces (client hot loop, bench)
* :mod:`dwpa_amd.help_crack` -- ``run_cracker`` replacement for help_crack.py
"""
from ._lib import DwpaError, load  # noqa: F401
from .m22000 import (BatchJobs, check_batch, check_key_m22000, crack_files, device_count, group_by_essid,  # noqa: F401
                     check_stats, hash_m22000, hc_unhex, init, parse_m22000, pbkdf2_pmk, rules_count, rules_count_ex,
                     rules_expand, Scan)

__all__ = ["DwpaError", "load", "BatchJobs", "check_key_m22000", "check_batch", "pbkdf2_pmk", "hc_unhex", "hash_m22000",
           "crack_files", "rules_count", "rules_count_ex", "check_stats", "rules_expand", "device_count", "Scan",
           "parse_m22000", "group_by_essid", "init"]
