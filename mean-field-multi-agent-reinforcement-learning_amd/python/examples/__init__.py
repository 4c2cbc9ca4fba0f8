"""Drop-in `examples` package (only `examples.ising_model` is provided).

A regular package on purpose: the reference keeps `examples/` as a namespace package next to
main_MFQ_Ising.py, and a regular package anywhere on sys.path wins over namespace portions, so
`examples.ising_model` resolves here even when the script runs from the reference's directory."""
