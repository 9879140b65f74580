"""Data layer: reference-format .mat datasets, synthetic DAS generator, HBM-resident datasets."""
from .mat_dataset import (DataCollector, Dataset_mat_MTL, DatasetDisk, Datasetram, add_gaussian, data_process,
                          measured_snr, split_category)
from .synthetic import DeviceDataset, generate, write_mat_tree
