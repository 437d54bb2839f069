"""Configuration constants (mirror of the reference's config.py:15-39, same names/values).

They are passed to the kernels as scalar arguments; nothing is read from the
environment.  ``TIE_TOLERANCE`` and the validation limits are unused by the reference
as well and are kept only for import compatibility.
"""

# Cold-start defaults (config.py:17-18)
DEFAULT_RELIABILITY = 0.50
DEFAULT_CONFIDENCE = 0.25

# Reliability update constraint (config.py:22)
MAX_UPDATE_STEP = 0.10

# Tie-breaking tolerance (config.py:26; unused by the reference)
TIE_TOLERANCE = 1e-9

# Decay (config.py:30-31)
DECAY_HALF_LIFE_DAYS = 30
DECAY_MINIMUM = 0.10

# Schema versioning (config.py:34)
SCHEMA_VERSION = "1.0.0"

# Validation limits (config.py:37-39; unused by the reference)
MIN_SOURCE_ID_LENGTH = 1
MAX_SOURCE_ID_LENGTH = 256
MAX_SIGNALS_PER_REQUEST = 1000

# Learning rate applied before capping (reliability.py:34)
BASE_LEARNING_RATE = 0.15
