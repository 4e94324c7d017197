"""End-to-end training recipes — one per reference script, each runnable
sequentially (one executor) or data-parallel on N MI355X executors via Distributor:

  mlp         distributed_multilayer_perceptron.py / pytorch_multilayer_perceptron.py
  cnn         distributed_cnn.py / pytorch_cnn.py
  lstm        distributed_lstm.py / pytorch_lstm.py
  translator  pytorch_machine_translator.py (+ transformer.py), data-parallel as well
  mllib_mlp   mllib_multilayer_perceptron_classifier.py

``python -m sparkmi.recipes.<name> --world 8 --epochs 3 ...`` or ``recipes.<name>.main(argv)``.
"""
