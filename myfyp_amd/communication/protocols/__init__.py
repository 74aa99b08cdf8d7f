"""Transport protocols behind one ``CommunicationProtocol`` contract."""
