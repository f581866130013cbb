"""Domain-adaptation methods on the detector: DAF (lib/DAF), MAF (lib/MAF), ATF (lib/ATF)."""
