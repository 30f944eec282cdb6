"""ollama-operator for AMD Instinct MI355X (gfx950): an API-compatible `ollama.ayaka.io/v1` Model
operator plus a from-scratch Ollama-REST inference server whose hot ops are hand-written CDNA4 HIP
kernels. See README.md and SURVEY.md."""

__version__ = "0.1.0"
