from .constants import FileType, GGMLType, ValueType, BLOCK_GEOMETRY, QK_K, tensor_nbytes  # noqa: F401
from .reader import GGUFError, GGUFFile, TensorInfo, read_gguf  # noqa: F401
from .writer import GGUFWriter  # noqa: F401
