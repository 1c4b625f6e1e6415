"""Drop-in replacements for the reference's denoising_model/ GP modules."""
