"""dynolog_amd.utils"""
