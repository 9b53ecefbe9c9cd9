"""lac_amd -- MI355X-native arithmetic coder with lac's predictor->coder surface."""
