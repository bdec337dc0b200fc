"""Model families: Llama-3 text generation and Stable Diffusion image generation."""
