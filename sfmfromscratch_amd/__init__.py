"""sfmfromscratch_amd — MI355X-native detect + describe + match stage of reesque/SfmFromScratch."""
