"""MI355X training payloads the example Crons schedule (``examples/mi355x``).

Standard library + PyTorch-ROCm only, so ``Dockerfile.payload`` can ship them on the ROCm
PyTorch base image without the operator's own dependencies.
"""
