"""Model zoo: reference Transformer (autograd), native HIP-path models (GPT-2, Llama-3, reference)."""
