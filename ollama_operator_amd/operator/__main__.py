from .controller import main

main()
