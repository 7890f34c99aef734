"""expecto_amd -- MI355X-native ExPecto chromatin-effect engine (Beluga hot path).

Heavy pieces (the HIP library, torch) load lazily so that pure-host utilities
(``synthetic``, ``encode``, ``genome``, ``h5``) import without a GPU.
"""
__version__ = "0.1.0"
