extern "C" __attribute__((visibility("default"))) const char* drpo_build_digest(void) { return "f476bbe94df44933ff5a06f0931a19117d8ae43c5fb93d226a18e8ea5814ea59"; }
