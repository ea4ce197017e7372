from dislib_amd.data.classes import Dataset, Subset
from dislib_amd.data.base import (load_data, load_libsvm_file,
                                  load_libsvm_files, load_txt_file,
                                  load_txt_files)

__all__ = ['Dataset', 'Subset', 'load_data', 'load_libsvm_file',
           'load_libsvm_files', 'load_txt_file', 'load_txt_files']
