"""mtl_das_pytorch_amd: MI355X-native multi-task DAS training framework."""
__version__ = "0.1.0"
