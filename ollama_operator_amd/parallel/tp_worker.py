"""Entry point of a tensor-parallel worker rank (spawned by `ollama serve` with OMX_TP > 1)."""
from .tp import worker_main

if __name__ == "__main__":
    worker_main()
